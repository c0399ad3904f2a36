#!/bin/bash
# Round 6, call 4: the GPU suite on the default build, then on the
# VR_EXPERIMENTS build (the fenced layouts / schedules re-tested), and config 5
# at N = 8 per-rank rehearsals: bands + compositor (the default) against
# weighted row ranges where rank 0 renders a reduced share beside its assembly.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c4
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 120 --timeout-method thread \
    > $O/gpu_suite.log 2>&1; rc=$?
tail -3 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 1,8 --streams 2 --frames 100 --rounds 3 \
    > $O/c5_default.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/c5_default.txt; [ $rc -eq 0 ] || exit $rc
for pct in 30 50 70; do
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 8 --streams 2 --frames 100 --rounds 3 \
    --partition rows --compositor off --opt row_first_pct=$pct > $O/c5_rows_pct$pct.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/c5_rows_pct$pct.txt; [ $rc -eq 0 ] || exit $rc
done
# the VR_EXPERIMENTS build over the default one, in this box's copy only
cp volumetricrenderer_amd/libvr_experiments.so volumetricrenderer_amd/libvr.so
cp volumetricrenderer_amd/libvr_shard_experiments.so volumetricrenderer_amd/libvr_shard.so
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 120 --timeout-method thread \
    > $O/gpu_suite_experiments.log 2>&1; rc=$?
tail -3 $O/gpu_suite_experiments.log; exit $rc
