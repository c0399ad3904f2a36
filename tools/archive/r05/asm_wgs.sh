#!/bin/bash
# rank 0's assembly grid size at N = 8 (config 5, solo rank 0)
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for w in 1024 2048 768 1024 2048; do
  echo "== VR_ASM_WGS=$w"
  VR_ASM_WGS=$w timeout -k 10 200 python -u tools/band_scaling.py --native --ns 8 --streams 2 --frames 100 --rounds 3 \
      > $O/aw.txt 2>&1 || { cat $O/aw.txt; exit 3; }
  grep -v amdgpu.ids $O/aw.txt | grep "N=8"
done
