#!/bin/bash
# Round 2 experiment 1: per-wave timeline of the 512^3 frame (critical path vs
# throughput) with wave priority and step split; zpair vs brick4832 at 512^3.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"; export TMPDIR=/tmp
TL="env VR_LIB=volumetricrenderer_amd/libvr_tl.so timeout -k 10 180 python -u tools/timeline.py"
for cfg in "--reps 1" "--reps 1 --opt prio=28" "--reps 1 --opt prio=36" "--reps 1 --opt prio=20" "--reps 1 --split 2" "--reps 1"; do
  $TL $cfg >> "$OUT/tl_512.log" 2>&1 || { tail "$OUT/tl_512.log"; exit 3; }
done
grep -v amdgpu.ids "$OUT/tl_512.log"
timeout -k 10 300 python -u tools/layout_sweep.py --sizes 512 --variants 12:5:2:4,7:5:2:4 --rounds 5 --no-check > "$OUT/sweep_zpair.log" 2>&1 || { tail "$OUT/sweep_zpair.log"; exit 4; }
grep -v amdgpu.ids "$OUT/sweep_zpair.log" | head -4
