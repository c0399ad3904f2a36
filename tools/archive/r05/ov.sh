#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_distributed.py -q -x --tb=short --timeout 120 --timeout-method thread \
    > $O/ov_dist.log 2>&1; rc=$?
tail -1 $O/ov_dist.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 1,2,4,8 --streams 2 --frames 100 --rounds 3 \
    > $O/ov_c5.txt 2>&1 || { cat $O/ov_c5.txt; exit 3; }
grep -v amdgpu.ids $O/ov_c5.txt
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 1,2,4,8 --streams 2 --size 128 --width 3840 \
    --height 2160 --steps 256 --frames 40 --rounds 3 > $O/ov_c4.txt 2>&1 || { cat $O/ov_c4.txt; exit 4; }
grep -v amdgpu.ids $O/ov_c4.txt
