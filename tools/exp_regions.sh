#!/bin/bash
# Regions vs rings schedule sweep.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "regions or schedules or off_centre" > $OUT/pytest_regions.log 2>&1 || { echo tests fail; tail -20 $OUT/pytest_regions.log; exit 1; }
tail -2 $OUT/pytest_regions.log
sw() { timeout -k 10 300 python tools/layout_sweep.py --rounds 5 --frames 10 "$@" > $OUT/sw.log 2>&1 || { echo sweep fail "$@"; tail $OUT/sw.log; exit 1; }; grep median $OUT/sw.log; }
sw --sizes 512 --variants 2:4:2,2:5:2:2,2:5:2:3,2:5:2:8,2:5:3:2
sw --sizes 128 --variants 5:4:2,5:5:2:2,5:5:2:4,5:5:2:8,5:5:1:2,5:5:3:4
sw --sizes 128 --width 3840 --height 2160 --steps 256 --variants 5:4:2,5:5:2:2,5:5:2:4,5:5:1:4
echo ok
