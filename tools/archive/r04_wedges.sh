#!/bin/bash
# round 4: finer wedges (long tiles spread over more XCDs) at N = 1, 2, 4, 8
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
V="-1:0:0:8,-1:0:0:16,-1:0:0:32,-1:0:0:64,-1:0:0:8"
timeout -k 10 400 python -u tools/band_scaling.py --all-ranks --variants="$V" > gpurun_out/r04_wedges_c5.txt 2>&1 || { tail gpurun_out/r04_wedges_c5.txt; exit 1; }
grep "rank-0" gpurun_out/r04_wedges_c5.txt
timeout -k 10 400 python -u tools/band_scaling.py --all-ranks --size 128 --width 3840 --height 2160 --steps 256 --variants="$V" > gpurun_out/r04_wedges_c4.txt 2>&1 || { tail gpurun_out/r04_wedges_c4.txt; exit 1; }
grep "rank-0" gpurun_out/r04_wedges_c4.txt
