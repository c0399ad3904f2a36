#!/bin/bash
# occupancy A/B of the primary procedural marches after the phased density
set -o pipefail
cd "$(dirname "$0")/../../.."
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/r05
L=volumetricrenderer_amd
LIBS="$L/libvr.so $L/libvr_w5.so $L/libvr_w3.so" CONFIGS="cloud cloud_shadow" ROUNDS=3 STEPS=30 \
    timeout -k 10 600 bash tools/abn.sh > gpurun_out/r05/ab_waves2.txt 2>&1; rc=$?
cat gpurun_out/r05/ab_waves2.txt; exit $rc
