#!/bin/bash
# layout builder: parity (every layout, config-5 bands) and kernel times at 512^3
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "every_layout or config5 or generator" > "$OUT/pytest_build.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_build.log"; [ $rc -ne 0 ] && exit $rc
rm -rf "$OUT/gen512"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/gen512" -o run --output-format csv -- python3 tools/prof_case.py --size 512 --frames 2 > "$OUT/gen512.log" 2>&1 || { tail "$OUT/gen512.log"; exit 5; }
find "$OUT/gen512" -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1-5 | head -20
