#!/bin/bash
# round 5, call 7: where a solo 1/8-frame period goes (kernel trace of the
# native loop, exchange on the render streams), config 4 with the exchange on
# the render streams, and the deferred-shadow primary march's unroll /
# occupancy A/B (config 3)
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_solo8 -o solo8 -- \
    python -u tools/band_scaling.py --native --ns 8 --streams 2 --frames 100 --rounds 2 --on-render \
    > $O/c7_prof_solo8.txt 2>&1 || { tail -20 $O/c7_prof_solo8.txt; exit 2; }
grep -v amdgpu.ids $O/c7_prof_solo8.txt | tail -3
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 1,4,8 --size 128 --width 3840 --height 2160 --steps 256 \
    --frames 40 --rounds 3 --on-render > $O/c7_native_c4_onr.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/c7_native_c4_onr.txt; [ $rc -eq 0 ] || exit 4
L=volumetricrenderer_amd
LIBS="$L/libvr_base.so $L/libvr.so $L/libvr_v4.so $L/libvr_v5.so $L/libvr_v6.so" CONFIGS="cloud_shadow" ROUNDS=3 STEPS=30 \
    timeout -k 10 700 bash tools/abn.sh > $O/c7_ab_defer.txt 2>&1; rc=$?
cat $O/c7_ab_defer.txt; exit $rc
