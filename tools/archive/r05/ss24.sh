#!/bin/bash
# split K / tiles per wave at N = 2 and 4 after empty-tile fill (config 5)
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for o in "" "--opt split=1" "--opt split=2" "--opt split=4" "--opt tiles_per_wave=1" "--opt tiles_per_wave=4"; do
  echo "== ${o:-default}"
  timeout -k 10 200 python -u tools/band_scaling.py --native --all-ranks --ns 2,4 --streams 2 --frames 100 --rounds 3 $o \
      > $O/ss24.txt 2>&1 || { cat $O/ss24.txt; exit 3; }
  grep -v amdgpu.ids $O/ss24.txt | grep "N=\|per rank"
done
