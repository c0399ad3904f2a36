#!/bin/bash
# Round 6, call 5: config 4 at N = 8 with row ranges from the makespan model
# (tools/row_cost_model.py --candidates) against the default split, then the GPU
# suite on the VR_EXPERIMENTS build (the fenced layouts / schedules re-tested).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c5
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
C4="--native --all-ranks --streams 3 --frames 40 --rounds 3 --size 128 --width 3840 --height 2160 --steps 256"
timeout -k 10 400 python -u tools/band_scaling.py $C4 --ns 8 --partition rows \
    --rows 0,704,848,960,1064,1168,1288,1432,2160 --rows 0,696,856,976,1064,1152,1272,1456,2160 \
    --rows 0,704,856,968,1064,1160,1280,1448,2160 --rows 0,664,816,944,1056,1168,1312,1496,2160 \
    --rows 0,704,848,960,1064,1168,1288,1432,2160 > $O/c4_rows.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/c4_rows.txt; [ $rc -eq 0 ] || exit $rc
cp volumetricrenderer_amd/libvr_experiments.so volumetricrenderer_amd/libvr.so
cp volumetricrenderer_amd/libvr_shard_experiments.so volumetricrenderer_amd/libvr_shard.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 120 --timeout-method thread \
    > $O/gpu_suite_experiments.log 2>&1; rc=$?
tail -3 $O/gpu_suite_experiments.log; exit $rc
