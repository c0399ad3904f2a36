#!/bin/bash
# round 4, final code: focused parity (region orders, spinning, split rays),
# the round evidence (bench line + rocprof + spin lines + per-rank bands),
# then the GPU suite on the default build and on the VR_EXPERIMENTS build
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --tb=short --timeout 120 --timeout-method thread \
    -k "region_order or spinning or split_rays or one_eighth or outlive" > gpurun_out/r04_final_dbg.log 2>&1 || { tail -30 gpurun_out/r04_final_dbg.log; exit 1; }
tail -1 gpurun_out/r04_final_dbg.log
bash tools/archive/r04_round.sh || exit 2
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --tb=short --timeout 120 --timeout-method thread > gpurun_out/r04_pytest.log 2>&1
rc=$?
tail -2 gpurun_out/r04_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
cp volumetricrenderer_amd/libvr_exp.so volumetricrenderer_amd/libvr.so
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --tb=short --timeout 120 --timeout-method thread > gpurun_out/r04_pytest_exp.log 2>&1
rc=$?
tail -2 gpurun_out/r04_pytest_exp.log
exit $rc
