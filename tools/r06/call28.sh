#!/bin/bash
# Round 6, call 28: 8-rank defaults for every frame size (serpentine band sets,
# rank 0 compositing + lead rows): the frame-loop GPU tests, then the per-rank
# frame streams of configs 5 and 4 at N = 1, 2, 4, 8 with the defaults.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c28
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu --maxfail 5 -q --tb=short --timeout 120 --timeout-method thread \
    -k "distributed or loopback or config4 or lead or serpentine or solo" > $O/gpu_loop.log 2>&1; rc=$?
tail -3 $O/gpu_loop.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/band_scaling.py --native --all-ranks --ns 1,2,4,8 --streams 2 --frames 100 --rounds 3 \
    > $O/native_c5.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/native_c5.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/band_scaling.py --native --all-ranks --ns 1,2,4,8 --streams 3 --size 128 --width 3840 \
    --height 2160 --steps 256 --frames 40 --rounds 3 > $O/native_c4.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/native_c4.txt; exit $rc
