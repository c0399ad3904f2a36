#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for br in 16 32 64 136; do
  echo "== c4 band_rows $br"
  timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 8 --streams 2 --size 128 --width 3840 --height 2160 \
      --steps 256 --frames 40 --rounds 3 --band-rows $br > $O/br.txt 2>&1 || { cat $O/br.txt; exit 3; }
  grep -v amdgpu.ids $O/br.txt | grep -A1 "N="
done
for br in 16 32 64; do
  echo "== c5 band_rows $br"
  timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 8 --streams 2 \
      --frames 100 --rounds 3 --band-rows $br > $O/br.txt 2>&1 || { cat $O/br.txt; exit 3; }
  grep -v amdgpu.ids $O/br.txt | grep -A1 "N="
done
