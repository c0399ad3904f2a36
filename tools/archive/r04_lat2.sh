#!/bin/bash
# lat sweep (configs 5 and 4, per rank, N = 1, 2, 4, 8), then the abort hunt
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
V="-1:0:0:0:0"
for k in 1 2 4 8; do for d in 2 3 4; do V="$V,-1:0:$k:0:$d"; done; done
timeout -k 10 300 python -u tools/band_scaling.py --all-ranks --variants="$V" > gpurun_out/r04_lat_c5.txt 2>&1 || { tail gpurun_out/r04_lat_c5.txt; exit 1; }
grep "rank-0" gpurun_out/r04_lat_c5.txt
timeout -k 10 300 python -u tools/band_scaling.py --all-ranks --size 128 --width 3840 --height 2160 --steps 256 --variants="$V" > gpurun_out/r04_lat_c4.txt 2>&1 || { tail gpurun_out/r04_lat_c4.txt; exit 1; }
grep "rank-0" gpurun_out/r04_lat_c4.txt
bash tools/archive/r04_abort.sh
