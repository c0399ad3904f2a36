#!/bin/bash
# round 4: schedule knobs under region_order 2 (the new default), per rank at
# N = 1, 2, 4, 8: split K, tiles per wave, wedges per XCD, supertile
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
V="-1:0:0,-1:0:2,-1:0:4,-1:0:8,-1:1:0,-1:3:0,-1:0:0:2,-1:0:0:8"
for cfg in c5 c4; do
  A=""; [ $cfg = c4 ] && A="--size 128 --width 3840 --height 2160 --steps 256"
  timeout -k 10 400 python -u tools/band_scaling.py --all-ranks $A --variants="$V" > gpurun_out/r04_tune_$cfg.txt 2>&1 || { tail gpurun_out/r04_tune_$cfg.txt; exit 1; }
  grep "rank-0" gpurun_out/r04_tune_$cfg.txt | grep -E "N=1|N=8"
  for st in 1 4; do
    timeout -k 10 300 python -u tools/band_scaling.py --all-ranks $A --opt supertile=$st > gpurun_out/r04_tune_${cfg}_st$st.txt 2>&1 || { tail gpurun_out/r04_tune_${cfg}_st$st.txt; exit 1; }
    grep "rank-0" gpurun_out/r04_tune_${cfg}_st$st.txt
  done
done
