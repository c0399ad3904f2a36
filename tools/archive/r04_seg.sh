#!/bin/bash
# round 4: ray segments (option segment) -- parity first, then the per-rank
# sweep of L at N = 1, 2, 4, 8 (configs 5 and 4), then the GPU suite
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v -s -x --tb=short --timeout 120 --timeout-method thread \
    -k "segments or one_eighth or outlive" > gpurun_out/r04_seg_dbg.log 2>&1
rc=$?
grep -E "PASSED|FAILED|Error|error|assert" gpurun_out/r04_seg_dbg.log | head -40
if [ $rc -ne 0 ]; then echo "focused pytest rc=$rc: stopping"; tail -30 gpurun_out/r04_seg_dbg.log; exit $rc; fi
V="-1:0:0:0:0:0"
for L in 8 16 24 32 48; do V="$V,-1:0:0:0:0:$L"; done
timeout -k 10 400 python -u tools/band_scaling.py --all-ranks --variants="$V" > gpurun_out/r04_seg_c5.txt 2>&1 || { tail gpurun_out/r04_seg_c5.txt; exit 1; }
grep "rank-0" gpurun_out/r04_seg_c5.txt
timeout -k 10 400 python -u tools/band_scaling.py --all-ranks --size 128 --width 3840 --height 2160 --steps 256 --variants="$V" > gpurun_out/r04_seg_c4.txt 2>&1 || { tail gpurun_out/r04_seg_c4.txt; exit 1; }
grep "rank-0" gpurun_out/r04_seg_c4.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -q -s -rf --tb=short --timeout 120 --timeout-method thread \
    > gpurun_out/r04_pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r04_pytest.log
exit $rc
