#!/bin/bash
# brick4 vs brick5, interleaved in one process per size.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python tools/layout_sweep.py --rounds 6 --frames 10 --sizes 512,384,200 --variants ${VARIANTS:-2:5:2:2,6:5:2:2,6:5:1:2,6:4:2} > $OUT/sw.log 2>&1 || { echo sweep fail; tail $OUT/sw.log; exit 1; }
grep median $OUT/sw.log
