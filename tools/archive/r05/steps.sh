#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u tools/band_scaling.py --native --all-ranks --streams 2 --size 128 --width 3840 --height 2160 \
    --steps 256 --frames 40 --rounds 2 --partition rows \
    --rows 0,704,848,960,1064,1168,1288,1432,2160 \
    --rows 0,704,848,960,1064,1176,1288,1432,2160 \
    --rows 0,704,848,960,1064,1184,1288,1432,2160 \
    --rows 0,704,848,960,1064,1168,1280,1432,2160 \
    --rows 0,704,848,960,1064,1168,1296,1432,2160 > $O/steps.txt 2>&1 || { cat $O/steps.txt; exit 3; }
grep -v amdgpu.ids $O/steps.txt
