#!/bin/bash
# round 5, call 1: the two-render-stream shard (parity), per-rank frame
# streams 1 vs 2 render streams (configs 5 and 4), the default bench line
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_distributed.py -q -x --tb=short --timeout 120 --timeout-method thread > $O/c1_dist.log 2>&1; rc=$?
tail -3 $O/c1_dist.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --frames 100 --rounds 3 > $O/c1_native_c5.txt 2>&1; rc=$?
cat $O/c1_native_c5.txt; [ $rc -eq 0 ] || exit 2
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --size 128 --width 3840 --height 2160 --steps 256 --frames 40 --rounds 3 > $O/c1_native_c4.txt 2>&1; rc=$?
cat $O/c1_native_c4.txt; [ $rc -eq 0 ] || exit 3
timeout -k 10 600 python -u bench.py > $O/c1_bench.json 2> $O/c1_bench.err; rc=$?
tail -c 3000 $O/c1_bench.json; [ $rc -eq 0 ] || { tail -20 $O/c1_bench.err; exit 4; }
