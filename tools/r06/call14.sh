#!/bin/bash
# Round 6, call 14: config 5 at N = 8 (lead rows, 2 streams): lanes per ray
# (vr option split) 0 = auto, 1, 2, 4, 8.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c14
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for sp in 0 1 2 4 8; do
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 8 --streams 2 --frames 100 --rounds 3 \
    --opt split=$sp > $O/c5_n8_split$sp.txt 2>&1; rc=$?
echo "split $sp"; grep -v amdgpu.ids $O/c5_n8_split$sp.txt | tail -2; [ $rc -eq 0 ] || exit $rc
done
