#!/bin/bash
# Round 6, call 21: with serpentine band sets, rank 0's share.  Config 5 per-rank
# frame streams at N = 2, 4, 8: the default (compositor from 8 ranks, lead at
# 40 %) against rank 0 as a compositor with lead rows at 40-95 % of a renderer,
# two interleaved rounds.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c21
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for round in 1 2; do
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 2,4,8 --streams 2 --frames 100 --rounds 3 \
    > $O/c5_default.txt 2>&1; rc=$?
echo "round $round default"; grep -A1 "slowest" $O/c5_default.txt | grep -v "^--"; [ $rc -eq 0 ] || exit $rc
for p in 40 60 80 95; do
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 2,4,8 --streams 2 --frames 100 --rounds 3 \
    --compositor on --lead-pct $p > $O/c5_lead$p.txt 2>&1; rc=$?
echo "round $round compositor lead $p"; grep -A1 "slowest\|lead rows" $O/c5_lead$p.txt | grep -v "^--"; [ $rc -eq 0 ] || exit $rc
done
done
