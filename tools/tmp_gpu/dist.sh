#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r05
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_distributed.py -q -x --tb=short --timeout 120 --timeout-method thread \
    > gpurun_out/r05/dist.log 2>&1; rc=$?
tail -3 gpurun_out/r05/dist.log; exit $rc
