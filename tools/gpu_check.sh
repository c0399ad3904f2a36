#!/bin/bash
# One gpurun session: smoke -> GPU tests -> bench -> rocprofv3 kernel trace.
# Every GPU step has its own time limit; a crash/abort/timeout ends the script.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
stop_if_fatal() {  # rc 0 = ok, 1 = test/assert failure: keep going; else stop
    if [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; then echo "FATAL rc=$1 in $2, stopping"; exit "$1"; fi
}
STEPS=${STEPS:-smoke,tests,bench,prof}
if [[ $STEPS == *smoke* ]]; then
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?
    echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"; stop_if_fatal $rc smoke
fi
if [[ $STEPS == *tests* ]]; then
    timeout -k 10 900 python -m pytest tests -m gpu -q ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1; rc=$?
    echo "pytest rc=$rc"; tail -15 "$OUT/pytest_gpu.log"; stop_if_fatal $rc pytest
fi
if [[ $STEPS == *bench* ]]; then
    timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.log" 2>&1; rc=$?
    echo "bench rc=$rc"; tail -3 "$OUT/bench.log"; stop_if_fatal $rc bench
fi
if [[ $STEPS == *offscreen* ]]; then
    timeout -k 10 120 ./tools/vr_offscreen --width 1920 --height 1080 --size 128 --frames 20 \
        --out "$OUT/frame_1080p.png" > "$OUT/offscreen.log" 2>&1; rc=$?
    echo "offscreen rc=$rc"; cat "$OUT/offscreen.log"; stop_if_fatal $rc offscreen
fi
if [[ $STEPS == *prof* ]]; then
    rm -rf "$OUT/prof"
    timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
        -- python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/prof.log" 2>&1; rc=$?
    echo "prof rc=$rc"; tail -2 "$OUT/prof.log"; stop_if_fatal $rc prof
fi
echo "gpu_check done"
