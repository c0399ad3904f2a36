#!/bin/bash
# Round 6, call 26: config 4 at N = 1, 2, 4, 8 (the final script's sequence),
# serpentine band sets with rank 0 as a compositor from 8 ranks and lead rows
# at 60 / 80 / 95 % of a renderer (call 25: row ranges and 40 %).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c26
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
C4="--native --all-ranks --ns 1,2,4,8 --streams 3 --size 128 --width 3840 --height 2160 --steps 256 --frames 40 --rounds 3"
for p in 60 80 95; do
timeout -k 10 400 python -u tools/band_scaling.py $C4 --partition bands --compositor on8 --lead-pct $p > $O/c4_lead$p.txt 2>&1; rc=$?
echo "config 4 lead $p"; grep -A1 "N=8 render\|lead rows" $O/c4_lead$p.txt | grep -v "^--"; [ $rc -eq 0 ] || exit $rc
done
