#!/bin/bash
# round 5, call 11: the procedural parity tests and Worley self-test after the
# offset-constant / min-init changes, their A/B against the previous build,
# and one kernel trace of the N=8 rank-0 solo loop with a single stream
# (the assembly kernel alone)
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x --tb=short --timeout 120 --timeout-method thread \
    -k "proc or worley or selftest or cloud or shadow" > $O/c11_tests.log 2>&1; rc=$?
tail -3 $O/c11_tests.log; [ $rc -eq 0 ] || exit $rc
L=volumetricrenderer_amd
LIBS="$L/libvr_prev.so $L/libvr.so" CONFIGS="cloud cloud_shadow" ROUNDS=3 STEPS=30 \
    timeout -k 10 500 bash tools/abn.sh > $O/c11_ab.txt 2>&1; rc=$?
cat $O/c11_ab.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_solo8d -o solo8 -- \
    python -u tools/band_scaling.py --native --ns 8 --streams 1 --frames 100 --rounds 2 --exchange comm \
    > $O/c11_prof_solo8.txt 2>&1 || { tail -20 $O/c11_prof_solo8.txt; exit 2; }
grep -v amdgpu.ids $O/c11_prof_solo8.txt | tail -2
