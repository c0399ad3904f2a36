#!/bin/bash
# Round 6, call 37: the GPU suite on the VR_EXPERIMENTS build after the
# serpentine band sets (the fenced layouts / schedules share the row mapping).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c37
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
cp volumetricrenderer_amd/libvr_experiments.so volumetricrenderer_amd/libvr.so
cp volumetricrenderer_amd/libvr_shard_experiments.so volumetricrenderer_amd/libvr_shard.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 120 --timeout-method thread \
    > $O/gpu_suite_experiments.log 2>&1; rc=$?
tail -3 $O/gpu_suite_experiments.log; exit $rc
