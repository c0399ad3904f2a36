#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 7,8 --streams 2 --frames 100 --rounds 3 \
    > $O/n7.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/n7.txt; exit $rc
