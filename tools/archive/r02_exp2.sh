#!/bin/bash
# Round 2 experiment 2: CORNERH (f16 {a, b-a} rows, fp32 index) parity and
# timing against CORNER8 at 128^3.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "every_layout or split_rays" > "$OUT/pytest_layouts.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_layouts.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/layout_sweep.py --sizes 128 --variants 5:5:2:4,14:5:2:4 --rounds 5 > "$OUT/sweep_ch_1080.log" 2>&1 || { tail "$OUT/sweep_ch_1080.log"; exit 4; }
grep -v amdgpu.ids "$OUT/sweep_ch_1080.log" | head -3
timeout -k 10 300 python -u tools/layout_sweep.py --sizes 128 --width 3840 --height 2160 --steps 256 --variants 5:5:2:4,14:5:2:4 --rounds 5 > "$OUT/sweep_ch_4k.log" 2>&1 || { tail "$OUT/sweep_ch_4k.log"; exit 5; }
grep -v amdgpu.ids "$OUT/sweep_ch_4k.log" | head -3
