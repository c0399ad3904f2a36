#!/bin/bash
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "every_layout" > "$OUT/pytest_l.log" 2>&1 || { tail "$OUT/pytest_l.log"; exit 2; }
tail -1 "$OUT/pytest_l.log"
timeout -k 10 300 python -u tools/band_scaling.py --size 128 --width 3840 --height 2160 --steps 256 --variants=-1:0:0:0:0,-1:0:0:0:1,-1:0:2:0:1,-1:1:0:0:1 > "$OUT/bands4k.log" 2>&1 || { tail "$OUT/bands4k.log"; exit 4; }
grep -v amdgpu "$OUT/bands4k.log"
timeout -k 10 300 python -u tools/band_scaling.py --size 128 --variants=-1:0:0:0:0,-1:0:0:0:1 > "$OUT/bands128.log" 2>&1 || { tail "$OUT/bands128.log"; exit 4; }
grep -v amdgpu "$OUT/bands128.log"
