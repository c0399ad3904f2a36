#!/bin/bash
# the full-suite abort in vr_render (test_wrap_mode_switch_at_the_margin after
# the earlier parity tests): the same order with output uncaptured, so the
# message printed before abort() is kept
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -s -v -x --tb=short --timeout 120 --timeout-method thread \
    > gpurun_out/r04_abort.log 2>&1
rc=$?
grep -nE "Memory access|fault|free\(\)|malloc|corrupt|double free|terminate|Assertion|error|Error" gpurun_out/r04_abort.log | grep -v "PASSED" | head -20
tail -5 gpurun_out/r04_abort.log
exit $rc
