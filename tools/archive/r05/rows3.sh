#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for m in "40 130 85" "40 130 70" "60 125 80" "40 140 80" "80 130 80"; do
  set -- $m
  echo "== row_setup $1 row_pow $2 row_first_pct $3"
  timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 8 --streams 2 --size 128 --width 3840 --height 2160 \
      --steps 256 --frames 40 --rounds 3 --partition rows --opt row_setup=$1 --opt row_pow=$2 --opt row_first_pct=$3 > $O/rows_c4.txt 2>&1 || { cat $O/rows_c4.txt; exit 3; }
  grep -v amdgpu.ids $O/rows_c4.txt | grep -A1 "N="
done
