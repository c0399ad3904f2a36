#!/bin/bash
# Round 6, call 27: config 4 at N = 1, 2, 4, 8 on one box, two interleaved
# rounds: row ranges at 8 ranks (the round-5 default) against serpentine band
# sets with rank 0 as a compositor from 8 ranks and lead rows at 80 %.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c27
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
C4="--native --all-ranks --ns 1,2,4,8 --streams 3 --size 128 --width 3840 --height 2160 --steps 256 --frames 40 --rounds 3"
for round in 1 2; do
for v in "rows:--partition auto" "lead80:--partition bands --compositor on8 --lead-pct 80"; do
name=${v%%:*}; args=${v#*:}
timeout -k 10 400 python -u tools/band_scaling.py $C4 $args > $O/c4_${name}_$round.txt 2>&1; rc=$?
echo "round $round config 4 $name"; grep -A1 "render_streams\|lead rows" $O/c4_${name}_$round.txt | grep -v "^--"; [ $rc -eq 0 ] || exit $rc
done
done
