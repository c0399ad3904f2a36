#!/bin/bash
# round 5, call 6: the shard tests (exchange on the render streams added),
# GPU-only per-rank frame period (gated queue) vs the live host-paced one,
# exchange on the comm stream vs on the render streams, configs 5 and 4;
# procedural A/B of the default build against round 4's
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_distributed.py -q -x --tb=short --timeout 120 --timeout-method thread > $O/c6_dist.log 2>&1; rc=$?
tail -3 $O/c6_dist.log; [ $rc -eq 0 ] || exit $rc
for g in 0 8; do for orr in "" "--on-render"; do
  timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 1,4,8 --frames 100 --rounds 3 --gate-ms $g $orr \
      > $O/c6_native_c5_g${g}${orr}.txt 2>&1 || { cat $O/c6_native_c5_g${g}${orr}.txt; exit 2; }
  cat $O/c6_native_c5_g${g}${orr}.txt | grep -v amdgpu.ids
done; done
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 1,4,8 --size 128 --width 3840 --height 2160 --steps 256 \
    --frames 40 --rounds 3 --gate-ms 15 > $O/c6_native_c4_gated.txt 2>&1; rc=$?
cat $O/c6_native_c4_gated.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit 4
L=volumetricrenderer_amd
LIBS="$L/libvr_base.so $L/libvr.so" CONFIGS="cloud cloud_shadow" ROUNDS=3 STEPS=30 \
    timeout -k 10 600 bash tools/abn.sh > $O/c6_ab_proc.txt 2>&1; rc=$?
cat $O/c6_ab_proc.txt; exit $rc
