#!/bin/bash
# Round 6, call 9: the GPU suite with rank 0's lead rows on by default for the
# compositor, the default bench line, and config 5 / config 4 per-rank
# rehearsals at N = 1, 2, 4, 8 with the defaults.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c9
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 120 --timeout-method thread \
    > $O/gpu_suite.log 2>&1; rc=$?
tail -3 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; rc=$?
tail -c 300 $O/bench.json; [ $rc -eq 0 ] || { tail $O/bench.err; exit $rc; }
timeout -k 10 400 python -u tools/band_scaling.py --native --all-ranks --ns 1,2,4,8 --streams 2 --frames 100 --rounds 3 \
    > $O/c5_native.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/c5_native.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/band_scaling.py --native --all-ranks --ns 1,2,4,8 --streams 3 --size 128 --width 3840 \
    --height 2160 --steps 256 --frames 40 --rounds 3 > $O/c4_native.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/c4_native.txt; exit $rc
