#!/bin/bash
# Round 6, call 19: deferred shadow chunks numbered across the frame (one partial
# chunk per frame, not per wave): the procedural GPU tests, then config 3 / 2
# against the previous build (libvr_ab.so), interleaved on one box.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c19
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 120 --timeout-method thread \
    -k "procedural or config3 or shadow or cloud" > $O/gpu_proc.log 2>&1; rc=$?
tail -2 $O/gpu_proc.log; [ $rc -eq 0 ] || exit $rc
LIBB=volumetricrenderer_amd/libvr_ab.so CONFIGS="cloud_shadow" ROUNDS=4 STEPS=40 bash tools/ab.sh
