#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for o in "--opt split=1" "--opt split=2" "--opt split=1 --opt tiles_per_wave=1" "--opt split=1 --opt tiles_per_wave=2"; do
  echo "== $o"
  timeout -k 10 200 python -u tools/band_scaling.py --native --ns 1 --streams 1 --frames 100 --rounds 3 $o \
      > $O/k2.txt 2>&1 || { cat $O/k2.txt; exit 3; }
  grep -v amdgpu.ids $O/k2.txt | grep "N="
done
