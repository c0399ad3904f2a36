#!/bin/bash
# round 5, call 10: the SLP vectoriser off (no lane-transposing moves around
# the lerps) A/B on every config; the shard tests with the exchange on the
# render streams as the default
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=volumetricrenderer_amd
LIBS="$L/libvr.so $L/libvr_noslp.so" CONFIGS="cloud cloud_shadow grid512 grid4k" ROUNDS=3 STEPS=30 \
    timeout -k 10 700 bash tools/abn.sh > $O/c10_ab_noslp.txt 2>&1; rc=$?
cat $O/c10_ab_noslp.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_distributed.py -q -x --tb=short --timeout 120 --timeout-method thread \
    > $O/c10_dist.log 2>&1; rc=$?
tail -3 $O/c10_dist.log; exit $rc
