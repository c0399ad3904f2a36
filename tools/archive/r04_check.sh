#!/bin/bash
# round 4, last check of the shipped libraries: smoke() and the GPU suite
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04_smoke.log 2>&1 || { tail -20 gpurun_out/r04_smoke.log; exit 1; }
tail -1 gpurun_out/r04_smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --tb=short --timeout 120 --timeout-method thread > gpurun_out/r04_pytest_last.log 2>&1
rc=$?
tail -2 gpurun_out/r04_pytest_last.log
exit $rc
