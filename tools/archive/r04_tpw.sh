#!/bin/bash
# round 4: tiles per wave and wedges per XCD for the whole config-5 / config-4
# frame under region_order 2, interleaved three times on one box
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
V="-1:0:0,-1:3:0,-1:4:0,-1:0:0:8,-1:3:0:8"
V="$V,$V,$V"
timeout -k 10 400 python -u tools/band_scaling.py --ns 1 --frames 40 --variants="$V" > gpurun_out/r04_tpw_c5.txt 2>&1 || { tail gpurun_out/r04_tpw_c5.txt; exit 1; }
grep "rank-0" gpurun_out/r04_tpw_c5.txt
timeout -k 10 400 python -u tools/band_scaling.py --ns 1,8 --frames 40 --all-ranks --variants="-1:0:0,-1:3:0,-1:0:0:8,-1:3:0:8" > gpurun_out/r04_tpw_c5n8.txt 2>&1 || { tail gpurun_out/r04_tpw_c5n8.txt; exit 1; }
grep "rank-0" gpurun_out/r04_tpw_c5n8.txt
timeout -k 10 400 python -u tools/band_scaling.py --ns 1 --frames 30 --size 128 --width 3840 --height 2160 --steps 256 --variants="$V" > gpurun_out/r04_tpw_c4.txt 2>&1 || { tail gpurun_out/r04_tpw_c4.txt; exit 1; }
grep "rank-0" gpurun_out/r04_tpw_c4.txt
