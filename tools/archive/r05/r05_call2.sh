#!/bin/bash
# round 5, call 2: smoke with the build id, the exception guard and the
# spinning / region tests, then the host cost per frame of the native loop
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/c2_smoke.log 2>&1; rc=$?
tail -3 $O/c2_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_distributed.py -q -x --tb=short --timeout 120 --timeout-method thread \
    -k "exception or spinning or region or solo or loopback or in_flight" > $O/c2_tests.log 2>&1; rc=$?
tail -3 $O/c2_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/host_frame 40 > $O/c2_host_frame.txt 2>&1; rc=$?
cat $O/c2_host_frame.txt; exit $rc
