#!/bin/bash
# round 5, call 20: per-rank frame streams rehearsed one rank's pipeline at a
# time (its streams on hardware queues of their own), configs 5 and 4
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u tools/band_scaling.py --native --all-ranks --ns 1,4,8 --streams 1,2 --frames 100 --rounds 3 \
    > $O/c20_native_c5.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/c20_native_c5.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/band_scaling.py --native --all-ranks --ns 1,8 --streams 2 --size 128 --width 3840 --height 2160 \
    --steps 256 --frames 40 --rounds 3 > $O/c20_native_c4.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/c20_native_c4.txt; exit $rc
