#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for o in "--opt split=1" "--opt split=2"; do
  echo "== c5 $o"
  timeout -k 10 200 python -u tools/band_scaling.py --native --all-ranks --ns 2 --streams 1,2 --frames 100 --rounds 3 $o \
      > $O/ss2.txt 2>&1 || { cat $O/ss2.txt; exit 3; }
  grep -v amdgpu.ids $O/ss2.txt | grep "N=\|per rank"
  echo "== c4 $o"
  timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 4,8 --streams 2 --size 128 --width 3840 \
      --height 2160 --steps 256 --frames 40 --rounds 3 $o > $O/ss2c4.txt 2>&1 || { cat $O/ss2c4.txt; exit 4; }
  grep -v amdgpu.ids $O/ss2c4.txt | grep "N=\|per rank"
done
