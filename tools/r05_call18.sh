#!/bin/bash
# round 5, call 18: per-rank frame periods at N = 6, 7, 8 (config 5), to size a
# compositor rank 0 (renderers at a 1/7 share, rank 0 assembling only)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 1,6,7,8 --streams 2 --frames 100 --rounds 3 \
    > $O/c18_native_c5_678.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/c18_native_c5_678.txt; exit $rc
