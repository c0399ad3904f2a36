#!/bin/bash
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "procedural" > "$OUT/pytest_proc.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_proc.log"; [ $rc -ne 0 ] && exit $rc
LIBB=volumetricrenderer_amd/libvr_base.so CONFIGS="cloud cloud_shadow" ROUNDS=3 bash tools/ab.sh
