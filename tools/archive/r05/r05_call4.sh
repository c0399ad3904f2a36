#!/bin/bash
# round 5, call 4: host cost per frame, procedural instruction-diet builds
# (A/B: base = HEAD before, v1 = loop-invariant density operands hoisted,
# v2 = + 4 octaves unrolled, v3 = v2 + occupancy-constrained), tests after
# the first-render retire events, per-rank frame streams
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 120 ./tools/host_frame 40 > $O/c4_host_frame.txt 2>&1; rc=$?
cat $O/c4_host_frame.txt; [ $rc -eq 0 ] || exit $rc
L=volumetricrenderer_amd
LIBS="$L/libvr_base.so $L/libvr_v1.so $L/libvr_v2.so $L/libvr_v3.so" CONFIGS="cloud cloud_shadow" ROUNDS=3 STEPS=30 \
    timeout -k 10 900 bash tools/abn.sh > $O/c4_ab_proc.txt 2>&1; rc=$?
cat $O/c4_ab_proc.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_distributed.py -q -x --tb=short --timeout 120 --timeout-method thread \
    -k "exception or spinning or region or solo or loopback or in_flight or procedural or outlive or launch_cache or in_place or one_rank" > $O/c4_tests.log 2>&1; rc=$?
tail -3 $O/c4_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --frames 100 --rounds 3 > $O/c4_native_c5.txt 2>&1; rc=$?
cat $O/c4_native_c5.txt; exit $rc
