#!/bin/bash
# round 5, call 6: GPU-only per-rank frame period (gated queue) vs the live
# host-paced one, configs 5 and 4; procedural A/B of the default build
# (primary fBm unrolled at 4 waves, hoisted operands) against round 4's
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 1,4,8 --frames 100 --rounds 3 --gate-ms 8 \
    > $O/c6_native_c5_gated.txt 2>&1; rc=$?
cat $O/c6_native_c5_gated.txt; [ $rc -eq 0 ] || exit 2
for sp in 1 2; do
  timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 8 --frames 100 --rounds 3 --gate-ms 8 --opt split=$sp \
      > $O/c6_native_c5_gated_split$sp.txt 2>&1 || { cat $O/c6_native_c5_gated_split$sp.txt; exit 3; }
  tail -2 $O/c6_native_c5_gated_split$sp.txt
done
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 1,4,8 --size 128 --width 3840 --height 2160 --steps 256 \
    --frames 40 --rounds 3 --gate-ms 15 > $O/c6_native_c4_gated.txt 2>&1; rc=$?
cat $O/c6_native_c4_gated.txt; [ $rc -eq 0 ] || exit 4
L=volumetricrenderer_amd
LIBS="$L/libvr_base.so $L/libvr.so" CONFIGS="cloud cloud_shadow" ROUNDS=3 STEPS=30 \
    timeout -k 10 600 bash tools/abn.sh > $O/c6_ab_proc.txt 2>&1; rc=$?
cat $O/c6_ab_proc.txt; exit $rc
