#!/bin/bash
# round 4: two earlier failures in detail, the whole GPU suite (latency-mode
# march, GPU region lists, frame-sized deferred scratch), then per-rank
# band-set timing of the latency-mode march against the split march at
# N = 1, 2, 4, 8 (configs 5, 4)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v -s --tb=short --timeout 120 --timeout-method thread \
    -k "spinning_camera_procedural or test_wrap_mode_switch_at_the_margin" > gpurun_out/r04_dbg.log 2>&1
rc=$?
grep -E "PASSED|FAILED|Error|error|assert" gpurun_out/r04_dbg.log | head -40
if [ $rc -gt 1 ]; then echo "focused pytest rc=$rc: stopping"; tail -30 gpurun_out/r04_dbg.log; exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --tb=line --timeout 120 --timeout-method thread \
    > gpurun_out/r04_pytest.log 2>&1
rc=$?
tail -25 gpurun_out/r04_pytest.log
if [ $rc -gt 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
V="-1:0:0:0:0"
for k in 1 2 4 8; do for d in 2 3 4; do V="$V,-1:0:$k:0:$d"; done; done
timeout -k 10 300 python -u tools/band_scaling.py --all-ranks --variants="$V" > gpurun_out/r04_lat_c5.txt 2>&1 || { tail gpurun_out/r04_lat_c5.txt; exit 1; }
grep "rank-0" gpurun_out/r04_lat_c5.txt
timeout -k 10 300 python -u tools/band_scaling.py --all-ranks --size 128 --width 3840 --height 2160 --steps 256 --variants="$V" > gpurun_out/r04_lat_c4.txt 2>&1 || { tail gpurun_out/r04_lat_c4.txt; exit 1; }
grep "rank-0" gpurun_out/r04_lat_c4.txt
