#!/bin/bash
# round 4: split march with one unit per idle tile -- parity, per-rank timing
# (configs 5 and 4), the default GPU suite, then the suite on the
# VR_EXPERIMENTS build (libvr_exp.so copied over libvr.so in this box's copy)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v -s -x --tb=short --timeout 120 --timeout-method thread \
    -k "split_rays or one_eighth or spinning or outlive or config4 or config5" > gpurun_out/r04_idle_dbg.log 2>&1
rc=$?
grep -cE "PASSED" gpurun_out/r04_idle_dbg.log; grep -E "FAILED|Error" gpurun_out/r04_idle_dbg.log | head
if [ $rc -ne 0 ]; then echo "focused pytest rc=$rc: stopping"; tail -30 gpurun_out/r04_idle_dbg.log; exit $rc; fi
timeout -k 10 300 python -u tools/band_scaling.py --all-ranks > gpurun_out/r04_idle_c5.txt 2>&1 || { tail gpurun_out/r04_idle_c5.txt; exit 1; }
grep "rank-0" gpurun_out/r04_idle_c5.txt
timeout -k 10 300 python -u tools/band_scaling.py --all-ranks --size 128 --width 3840 --height 2160 --steps 256 > gpurun_out/r04_idle_c4.txt 2>&1 || { tail gpurun_out/r04_idle_c4.txt; exit 1; }
grep "rank-0" gpurun_out/r04_idle_c4.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --tb=short --timeout 120 --timeout-method thread > gpurun_out/r04_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/r04_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
cp volumetricrenderer_amd/libvr_exp.so volumetricrenderer_amd/libvr.so
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --tb=short --timeout 120 --timeout-method thread > gpurun_out/r04_pytest_exp.log 2>&1
rc=$?
tail -3 gpurun_out/r04_pytest_exp.log
exit $rc
