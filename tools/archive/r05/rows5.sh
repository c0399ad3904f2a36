#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for o in "--opt split=0" "--opt split=2" "--opt split=2 --opt tiles_per_wave=1" "--opt split=0 --opt tiles_per_wave=1"; do
  echo "== rows $o"
  timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 8 --streams 2 --size 128 --width 3840 --height 2160 \
      --steps 256 --frames 40 --rounds 3 --partition rows $o > $O/rows5.txt 2>&1 || { cat $O/rows5.txt; exit 3; }
  grep -v amdgpu.ids $O/rows5.txt | grep -A1 "N="
done
