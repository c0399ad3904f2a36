#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for v in 0 1 0 1; do
  echo "== wave_prio=$v"
  timeout -k 10 200 python -u tools/band_scaling.py --native --ns 1,8 --streams 1,2 --frames 100 --rounds 3 --opt wave_prio=$v \
      > $O/pr.txt 2>&1 || { cat $O/pr.txt; exit 3; }
  grep -v amdgpu.ids $O/pr.txt | grep "N="
  timeout -k 10 200 python -u tools/band_scaling.py --native --ns 1 --streams 1 --size 128 --width 3840 --height 2160 \
      --steps 256 --frames 40 --rounds 3 --opt wave_prio=$v > $O/pr4.txt 2>&1 || { cat $O/pr4.txt; exit 4; }
  grep -v amdgpu.ids $O/pr4.txt | grep "N="
done
