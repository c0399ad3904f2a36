#!/bin/bash
# Round 6, call 29: band height with serpentine sets (16 rows, the default,
# against 24 and 32): per-rank frame streams of configs 5 and 4 at N = 1, 2, 4, 8
# with the defaults otherwise.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c29
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for br in 16 32 24; do
timeout -k 10 400 python -u tools/band_scaling.py --native --all-ranks --ns 1,2,4,8 --streams 2 --frames 100 --rounds 3 \
    --band-rows $br > $O/c5_br$br.txt 2>&1; rc=$?
echo "config 5 band rows $br"; grep -A1 "N=[248] render\|lead rows" $O/c5_br$br.txt | grep -v "^--"; [ $rc -eq 0 ] || exit $rc
done
for br in 16 32; do
timeout -k 10 400 python -u tools/band_scaling.py --native --all-ranks --ns 1,2,4,8 --streams 3 --size 128 --width 3840 \
    --height 2160 --steps 256 --frames 40 --rounds 3 --band-rows $br > $O/c4_br$br.txt 2>&1; rc=$?
echo "config 4 band rows $br"; grep -A1 "N=[248] render\|lead rows" $O/c4_br$br.txt | grep -v "^--"; [ $rc -eq 0 ] || exit $rc
done
