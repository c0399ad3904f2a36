#!/bin/bash
# round 5, call 12: the shadow pass's fBm loop without the loop-carried
# lattice prefetch (no rotation copies) A/B on config 3
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=volumetricrenderer_amd
LIBS="$L/libvr.so $L/libvr_nopf.so" CONFIGS="cloud_shadow" ROUNDS=4 STEPS=30 \
    timeout -k 10 500 bash tools/abn.sh > $O/c12_ab.txt 2>&1; rc=$?
cat $O/c12_ab.txt; exit $rc
