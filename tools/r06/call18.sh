#!/bin/bash
# Round 6, call 18: regions wedges per XCD 4 against 8 (the default) with frames
# in flight: config 5 and config 4 per-rank frame streams at N = 1 and 8, two
# interleaved rounds.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c18
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for round in 1 2; do
for w in 8 4; do
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 1,8 --streams 2 --frames 100 --rounds 3 \
    --opt wedges=$w > $O/c5_w$w.txt 2>&1; rc=$?
echo "round $round config 5 wedges $w"; grep "slowest" $O/c5_w$w.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 1,8 --streams 3 --size 128 --width 3840 \
    --height 2160 --steps 256 --frames 40 --rounds 3 --opt wedges=$w > $O/c4_w$w.txt 2>&1; rc=$?
echo "round $round config 4 wedges $w"; grep "slowest" $O/c4_w$w.txt; [ $rc -eq 0 ] || exit $rc
done
done
