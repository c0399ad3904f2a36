#!/bin/bash
# Round 6, call 23 (and 24, with the clock pre-warm): config 4 (4K x 256, 128^3) at N = 8 with serpentine band
# sets: row ranges (the default) against band sets, band sets with rank 0 as a
# compositor, and a compositor with lead rows at 40-80 % of a renderer.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/${CALL:-c23}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
C4="--native --all-ranks --ns 8 --streams 3 --size 128 --width 3840 --height 2160 --steps 256 --frames 40 --rounds 3"
for round in 1 2; do
for v in "rows:--partition rows" "bands:--partition bands --compositor off" "comp:--partition bands --compositor on --lead-pct 0" \
         "lead40:--partition bands --compositor on --lead-pct 40" "lead60:--partition bands --compositor on --lead-pct 60" \
         "lead80:--partition bands --compositor on --lead-pct 80"; do
name=${v%%:*}; args=${v#*:}
timeout -k 10 300 python -u tools/band_scaling.py $C4 $args > $O/c4_$name.txt 2>&1; rc=$?
echo "round $round config 4 $name"; grep -A1 "slowest\|lead rows" $O/c4_$name.txt | grep -v "^--"; [ $rc -eq 0 ] || exit $rc
done
done
