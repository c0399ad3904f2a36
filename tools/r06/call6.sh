#!/bin/bash
# Round 6, call 6: rank 0's lead rows (compositor + band sets below them):
# the new loopback / solo tests first, the whole GPU suite, then config 5 at
# N = 8 per-rank rehearsals with lead rows at 50 / 70 / 90 % of a share.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/${CALL:-c6}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py -m gpu -x -q --tb=short --timeout 120 \
    --timeout-method thread -k "lead or row_ranges_match" > $O/lead_tests.log 2>&1; rc=$?
tail -3 $O/lead_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 120 --timeout-method thread \
    > $O/gpu_suite.log 2>&1; rc=$?
tail -3 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 1,8 --streams 2 --frames 100 --rounds 3 \
    > $O/c5_default.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/c5_default.txt; [ $rc -eq 0 ] || exit $rc
for pct in 70 80 90 100; do
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 8 --streams 2 --frames 100 --rounds 3 \
    --lead-pct $pct > $O/c5_lead$pct.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/c5_lead$pct.txt; [ $rc -eq 0 ] || exit $rc
done
