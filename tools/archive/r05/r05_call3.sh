#!/bin/bash
# round 5, call 3: host cost per frame (pieces), the region / procedural /
# shard tests after the first-render retire events, per-rank frame streams
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 120 ./tools/host_frame 40 > $O/c3_host_frame.txt 2>&1; rc=$?
cat $O/c3_host_frame.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_distributed.py -q -x --tb=short --timeout 120 --timeout-method thread \
    -k "exception or spinning or region or solo or loopback or in_flight or procedural or outlive" > $O/c3_tests.log 2>&1; rc=$?
tail -3 $O/c3_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --frames 100 --rounds 3 > $O/c3_native_c5.txt 2>&1; rc=$?
cat $O/c3_native_c5.txt; exit $rc
