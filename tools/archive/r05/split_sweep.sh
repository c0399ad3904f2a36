#!/bin/bash
# the small share after empty-tile fill: split K and tiles per wave at N = 8 (compositor), config 5
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for o in "" "--opt split=2" "--opt split=8" "--opt tiles_per_wave=1" "--opt tiles_per_wave=2" "--opt tiles_per_wave=4" "--opt wedges=4"; do
  echo "== ${o:-default}"
  timeout -k 10 200 python -u tools/band_scaling.py --native --all-ranks --ns 8 --streams 2 --frames 100 --rounds 3 $o \
      > $O/ss.txt 2>&1 || { cat $O/ss.txt; exit 3; }
  grep -v amdgpu.ids $O/ss.txt | grep "N=8"
done
