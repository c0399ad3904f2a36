#!/bin/bash
# focused re-run of the two round-4 failures with full output
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v --tb=long --timeout 120 --timeout-method thread \
    -k "spinning_camera_procedural or test_wrap_mode_switch_at_the_margin" > gpurun_out/r04_dbg.log 2>&1
rc=$?
tail -80 gpurun_out/r04_dbg.log
exit $rc
