#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_distributed.py \
    -k "rebalance or row_ranges or solo" > $O/rb_tests.log 2>&1 || { tail -40 $O/rb_tests.log; exit 3; }
tail -1 $O/rb_tests.log
timeout -k 10 500 python -u tools/band_scaling.py --native --all-ranks --ns 8 --streams 2 --size 128 --width 3840 --height 2160 \
    --steps 256 --frames 40 --rounds 3 --partition rows --rebalance > $O/rb_c4.txt 2>&1 || { cat $O/rb_c4.txt; exit 3; }
grep -v amdgpu.ids $O/rb_c4.txt
