#!/bin/bash
# round 4: split_long as two launches (long tiles on a side stream with
# split_long_k lanes per ray) -- parity first, then the GPU suite, then the
# per-rank sweep at N = 1 and 8 (configs 5 and 4)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v -s -x --tb=short --timeout 120 --timeout-method thread \
    -k "split_long or outlive or spinning" > gpurun_out/r04_long_dbg.log 2>&1
rc=$?
grep -E "PASSED|FAILED|Error|error|assert" gpurun_out/r04_long_dbg.log | head -40
if [ $rc -ne 0 ]; then echo "focused pytest rc=$rc: stopping"; tail -30 gpurun_out/r04_long_dbg.log; exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -q -s -rf --tb=short --timeout 120 --timeout-method thread \
    > gpurun_out/r04_pytest.log 2>&1
rc=$?
tail -25 gpurun_out/r04_pytest.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
V="-1:0:0:0:0:0:4"
for s in 1 2 0; do for p in 30 50 70; do for k in 4 8; do V="$V,-1:0:$s:0:0:$p:$k"; done; done; done
timeout -k 10 400 python -u tools/band_scaling.py --all-ranks --ns 1,8 --variants="$V" > gpurun_out/r04_long_c5.txt 2>&1 || { tail gpurun_out/r04_long_c5.txt; exit 1; }
grep "rank-0" gpurun_out/r04_long_c5.txt
timeout -k 10 400 python -u tools/band_scaling.py --all-ranks --ns 1,8 --size 128 --width 3840 --height 2160 --steps 256 --variants="$V" > gpurun_out/r04_long_c4.txt 2>&1 || { tail gpurun_out/r04_long_c4.txt; exit 1; }
grep "rank-0" gpurun_out/r04_long_c4.txt
