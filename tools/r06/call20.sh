#!/bin/bash
# Round 6, call 20: serpentine band sets (vr_target.band_flip).  The GPU tests
# that cover band sets and the frame loop, then config 5 and config 4 per-rank
# frame streams at N = 8 (and 2, 4 for config 5) with the deal serpentine
# against plain, two interleaved rounds.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c20
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu --maxfail 10 -q --tb=short --timeout 120 --timeout-method thread \
    -k "serpentine or band or loopback or solo or assembl or distributed or lead" > $O/gpu_bands.log 2>&1; rc=$?
tail -3 $O/gpu_bands.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2; do
for sp in off on; do
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 1,2,4,8 --streams 2 --frames 100 --rounds 3 \
    --serpentine $sp > $O/c5_$sp.txt 2>&1; rc=$?
echo "round $round config 5 serpentine $sp"; grep -A1 "slowest" $O/c5_$sp.txt | grep -v "^--"; [ $rc -eq 0 ] || exit $rc
done
done
for sp in off on; do
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 1,8 --streams 3 --size 128 --width 3840 \
    --height 2160 --steps 256 --frames 40 --rounds 3 --partition bands --serpentine $sp > $O/c4_$sp.txt 2>&1; rc=$?
echo "config 4 bands serpentine $sp"; grep -A1 "slowest" $O/c4_$sp.txt | grep -v "^--"; [ $rc -eq 0 ] || exit $rc
done
