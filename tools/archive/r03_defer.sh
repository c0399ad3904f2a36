#!/bin/bash
# Config 3 deferred shadow rays (option shadow_defer): parity tests, then a
# same-box A/B against the in-wave compaction (interleaved), then a rocprofv3
# kernel trace of the deferred frame (time per pass).
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03defer; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "${TESTK:-deferred}" > $OUT/pytest.log 2>&1 || { echo tests fail; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in ${VARIANTS:-0 1}; do
    timeout -k 10 200 python -u bench.py --config ${CFG:-cloud_shadow} --opt shadow_defer=$v ${EXTRA:-} --no-cpu-baseline --steps 20 > $OUT/b.json 2> $OUT/b.err || { echo "bench $v fail"; tail -5 $OUT/b.err; exit 4; }
    python -c "import json;j=json.loads(open('$OUT/b.json').read());print('$r', 'shadow_defer=$v', j['ms_per_step'], j['kernel_ms_mean'], j['roofline']['frac'])"
  done
done | tee $OUT/ab.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o defer --output-format csv -- python3 -u bench.py --config ${CFG:-cloud_shadow} --opt shadow_defer=1 --no-cpu-baseline --steps 20 > $OUT/prof.log 2>&1 || { echo prof fail; tail -5 $OUT/prof.log; exit 5; }
find $OUT/prof -name "*kernel_stats.csv" -exec cp {} $OUT/defer_kernel_stats.csv \;
cut -d, -f1-8 $OUT/defer_kernel_stats.csv | head -12
