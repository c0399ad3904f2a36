#!/bin/bash
# Round-end validation: the whole GPU suite, smoke(), the default bench line and its
# rocprofv3 kernel statistics, the one-stream N = 1 line, per-rank frame streams (config 5 bands, config 4 row ranges)
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 120 --timeout-method thread \
    > $O/final_gpu_suite.log 2>&1; rc=$?
tail -2 $O/final_gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/final_smoke.log 2>&1; rc=$?
tail -2 $O/final_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/final_bench.json 2> $O/final_bench.err; rc=$?
tail -c 400 $O/final_bench.json; [ $rc -eq 0 ] || { tail $O/final_bench.err; exit $rc; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_final -o bench -- \
    python -u bench.py --no-cpu-baseline > $O/final_bench_prof.json 2> $O/final_bench_prof.err; rc=$?
[ $rc -eq 0 ] || { tail $O/final_bench_prof.err; exit $rc; }
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-other-configs --n1-loop sharder > $O/final_bench_sharder.json \
    2> $O/final_bench_sharder.err || exit 5
timeout -k 10 400 python -u tools/band_scaling.py --native --all-ranks --ns 1,2,4,8 --streams 2 --frames 100 --rounds 3 \
    > $O/final_native_c5.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/final_native_c5.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/band_scaling.py --native --all-ranks --ns 1,2,4,8 --streams 3 --size 128 --width 3840 \
    --height 2160 --steps 256 --frames 40 --rounds 3 > $O/final_native_c4.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/final_native_c4.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config grid4k --no-cpu-baseline > $O/final_bench_grid4k.json 2> $O/final_bench_grid4k.err; rc=$?
tail -c 300 $O/final_bench_grid4k.json; exit $rc
