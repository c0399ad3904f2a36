#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_distributed.py > $O/ns2_tests.log 2>&1 || { tail -40 $O/ns2_tests.log; exit 3; }
tail -1 $O/ns2_tests.log
timeout -k 10 500 python -u tools/band_scaling.py --native --all-ranks --ns 1,8 --streams 2,3,4 --frames 100 --rounds 3 > $O/ns2_c5.txt 2>&1 || { cat $O/ns2_c5.txt; exit 3; }
grep -v amdgpu.ids $O/ns2_c5.txt
timeout -k 10 500 python -u tools/band_scaling.py --native --all-ranks --ns 1,8 --streams 2,3,4 --size 128 --width 3840 --height 2160 \
    --steps 256 --frames 40 --rounds 3 > $O/ns2_c4.txt 2>&1 || { cat $O/ns2_c4.txt; exit 3; }
grep -v amdgpu.ids $O/ns2_c4.txt
timeout -k 10 500 python -u tools/band_scaling.py --native --all-ranks --ns 8 --streams 3,4 --size 128 --width 3840 --height 2160 \
    --steps 256 --frames 40 --rounds 3 --partition bands > $O/ns2_c4b.txt 2>&1 || { cat $O/ns2_c4b.txt; exit 3; }
grep -v amdgpu.ids $O/ns2_c4b.txt
