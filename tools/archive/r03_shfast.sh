#!/bin/bash
# Config 3 shadow-run fast path: parity, then same-box A/B against the previous
# build (libvr_base.so), configs 3 and 2.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03shfast; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "procedural or cloud or shadow or golden or spinning" > $OUT/pytest.log 2>&1 || { echo tests fail; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
LIBB=volumetricrenderer_amd/libvr_base.so CONFIGS="cloud_shadow cloud" ROUNDS=4 STEPS=20 timeout -k 10 600 bash tools/ab.sh | tee $OUT/ab.txt
