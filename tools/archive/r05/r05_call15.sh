#!/bin/bash
# round 5, call 15: the whole GPU suite on the current build, the procedural
# occupancy A/B (waves cap 4 / none / 5), the default bench line and its
# rocprofv3 kernel statistics
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 120 --timeout-method thread \
    > $O/c15_gpu_suite.log 2>&1; rc=$?
tail -3 $O/c15_gpu_suite.log; [ $rc -eq 0 ] || exit $rc
L=volumetricrenderer_amd
LIBS="$L/libvr.so $L/libvr_w0.so $L/libvr_w5.so" CONFIGS="cloud cloud_shadow" ROUNDS=3 STEPS=30 \
    timeout -k 10 600 bash tools/abn.sh > $O/c15_ab_waves.txt 2>&1; rc=$?
cat $O/c15_ab_waves.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/c15_bench.json 2> $O/c15_bench.err; rc=$?
tail -c 600 $O/c15_bench.json; [ $rc -eq 0 ] || { tail $O/c15_bench.err; exit $rc; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench -- \
    python -u bench.py --no-cpu-baseline > $O/c15_bench_prof.json 2> $O/c15_bench_prof.err; rc=$?
tail -c 300 $O/c15_bench_prof.json; exit $rc
