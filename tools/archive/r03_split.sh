#!/bin/bash
# split_long (march_regions_mixed) parity, then same-box A/B of the split
# threshold at config 5 (grid512) and config 4 (grid4k), interleaved.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03split; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "split or every_layout" > $OUT/pytest.log 2>&1 || { echo tests fail; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2 3; do
  for c in grid512 grid4k; do
    for v in ${PCTS:-0 40 60 75 90}; do
      timeout -k 10 200 python -u bench.py --config $c --opt split_long=$v --no-cpu-baseline --steps 40 > $OUT/b.json 2> $OUT/b.err || { echo "bench $c $v fail"; tail -5 $OUT/b.err; exit 4; }
      python -c "import json;j=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]);print('$r', '$c', '$v', j['ms_per_step'], j['kernel_ms_mean'], j['roofline']['frac'])"
    done
  done
done | tee $OUT/ab.txt
