#!/bin/bash
# Stale-order reuse of the procedural cost sort under a spinning camera:
# parity, then same-box A/B (sort_reuse 1 vs 0) of the spin bench, configs 2/3.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03sort; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "procedural or cloud or shadow or golden or spinning" > $OUT/pytest.log 2>&1 || { echo tests fail; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2 3; do
  for c in cloud cloud_shadow; do
    for v in ${RS:-0 1 2 4}; do
      timeout -k 10 200 python -u bench.py --config $c --spin --opt sort_reuse=$v --no-cpu-baseline --steps 64 > $OUT/b.json 2> $OUT/b.err || { echo "bench $c $v fail"; tail -5 $OUT/b.err; exit 4; }
      python -c "import json;j=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]);print('$r', '$c', 'sort_reuse=$v', j['ms_per_step'], j['kernel_ms_mean'], j['host_ms_per_frame'], j['roofline']['frac'])"
    done
  done
done | tee $OUT/ab.txt
