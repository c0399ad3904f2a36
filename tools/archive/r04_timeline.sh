#!/bin/bash
# round 4: per-wave / per-SIMD timeline of config 5's 1/8 share (rank 0's
# bands of 8) -- split 4 with 2 and 1 tiles per wave, one lane per ray, ray
# segments of 16 -- then the same for the whole frame (timing build libvr_tl.so)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 VR_LIB=$PWD/volumetricrenderer_amd/libvr_tl.so
run() { timeout -k 10 120 python3 -u tools/timeline.py --reps 2 "$@"; }
{ run --bands 8 --split 4 && run --bands 8 --split 4 --opt tiles_per_wave=1 && run --bands 8 --split 1 \
  && run --bands 1 --split 1; } > gpurun_out/r04_timeline.txt 2>&1
rc=$?
grep -E '^\{"opts' gpurun_out/r04_timeline.txt
exit $rc
