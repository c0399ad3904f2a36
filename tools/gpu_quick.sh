set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo tests fail; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.log 2>&1 || { echo bench fail; tail $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
for c in grid128 grid4k; do timeout -k 10 300 python bench.py --no-cpu-baseline --config $c > $OUT/bench_$c.log 2>&1 || exit 1; tail -1 $OUT/bench_$c.log | cut -c1-400; done
