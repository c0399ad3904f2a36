#!/bin/bash
# Uniform-channel skip: full GPU suite, then same-box A/B (uniform_skip 1 vs 0)
# at configs 5, 4 and 128^3 1080p, and the band scaling with the skip.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03uni; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo tests fail; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2 3; do
  for c in grid512 grid4k grid128; do
    for v in 1 0; do
      timeout -k 10 200 python -u bench.py --config $c --opt uniform_skip=$v --no-cpu-baseline --steps 40 > $OUT/b.json 2> $OUT/b.err || { echo "bench $c $v fail"; tail -5 $OUT/b.err; exit 4; }
      python -c "import json;j=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]);print('$r', '$c', 'uniform_skip=$v', j['config']['kernel'], j['ms_per_step'], j['kernel_ms_mean'], j['roofline']['frac'])"
    done
  done
done | tee $OUT/ab.txt
for v in 1 0; do
  timeout -k 10 200 python -u tools/band_scaling.py --size 512 --opt uniform_skip=$v 2>&1 | grep "N=" || exit 5
done | tee $OUT/bands.txt
