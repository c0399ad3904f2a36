#!/bin/bash
# Round 6, call 8: config 5 at N = 8 with 8-row bands (a finer interleave: half
# the per-period work gradient across the renderers), compositor alone and with
# rank 0's lead rows.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c8
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 8 --streams 2 --frames 100 --rounds 3 \
    --band-rows 8 > $O/c5_b8_default.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/c5_b8_default.txt; [ $rc -eq 0 ] || exit $rc
for pct in 40 50 60; do
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 8 --streams 2 --frames 100 --rounds 3 \
    --band-rows 8 --lead-pct $pct > $O/c5_b8_lead$pct.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/c5_b8_lead$pct.txt; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 8 --streams 2 --frames 100 --rounds 3 \
    --lead-pct 40 > $O/c5_b16_lead40.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/c5_b16_lead40.txt; exit $rc
