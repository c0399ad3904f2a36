#!/bin/bash
# Same-box A/B of several builds: bench.py with each of $LIBS (paths, the
# first is the reference), interleaved $ROUNDS times per config in $CONFIGS.
# Prints "round config lib ms_per_step kernel_ms frac".
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"; export TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-3}); do
  for c in ${CONFIGS:-cloud}; do
    for lib in $LIBS; do
      VR_LIB=$lib timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-other-configs --steps ${STEPS:-40} \
          ${BENCH_ARGS:-} > "$OUT/abn.log" 2> "$OUT/abn.err" || { tail "$OUT/abn.err"; exit 4; }
      python -c "import json;j=json.loads(open('$OUT/abn.log').read().strip().split(chr(10))[-1]);print('$r $c $(basename $lib)', j['ms_per_step'], j['kernel_ms_mean'], j['roofline']['frac'], flush=True)"
    done
  done
done
