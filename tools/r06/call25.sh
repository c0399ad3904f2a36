#!/bin/bash
# Round 6, call 25: config 4 at N = 1, 2, 4, 8 (the final script's sequence):
# row ranges at 8 ranks (the round-5 default) against serpentine band sets with
# rank 0 as a compositor and lead rows at 40 % of a renderer, two rounds.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c25
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
C4="--native --all-ranks --ns 1,2,4,8 --streams 3 --size 128 --width 3840 --height 2160 --steps 256 --frames 40 --rounds 3"
for round in 1 2; do
for v in "rows:--partition auto" "lead40:--partition bands --compositor on8 --lead-pct 40"; do
name=${v%%:*}; args=${v#*:}
timeout -k 10 400 python -u tools/band_scaling.py $C4 $args > $O/c4_$name.txt 2>&1; rc=$?
echo "round $round config 4 $name"; grep -A1 "N=8 render\|lead rows" $O/c4_$name.txt | grep -v "^--"; [ $rc -eq 0 ] || exit $rc
done
done
