#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/r05
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
VR_LIB=volumetricrenderer_amd/libvr_tlx.so timeout -k 10 200 python -u tools/timeline.py --reps 3 > gpurun_out/r05/tl1.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r05/tl1.txt | tail -40; [ $rc -eq 0 ] || exit $rc
VR_LIB=volumetricrenderer_amd/libvr_tlx.so timeout -k 10 200 python -u tools/timeline.py --reps 3 --opt empty_fill=0 > gpurun_out/r05/tl0.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r05/tl0.txt | tail -12; exit $rc
