#!/bin/bash
# Step-split rays: parity, then per-rank band times at N = 1..8.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "split" > $OUT/pt.log 2>&1 || { echo tests fail; tail -30 $OUT/pt.log; exit 1; }
tail -1 $OUT/pt.log
timeout -k 10 400 python tools/band_scaling.py --variants=${VARIANTS:--1:0:1,5:1:2,5:1:4,5:1:8,5:2:4,-1:0:0} > $OUT/bs.log 2>&1 || { echo bs fail; tail $OUT/bs.log; exit 1; }
grep schedule $OUT/bs.log
