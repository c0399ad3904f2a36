#!/bin/bash
# Round 2: full GPU suite, smoke, bench lines for the given configs.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_gpu.log"; echo "pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail "$OUT/smoke.log"; exit 3; }
tail -1 "$OUT/smoke.log"
for c in ${CONFIGS:-grid512}; do
  timeout -k 10 300 python -u bench.py --config $c > "$OUT/bench_$c.log" 2>&1 || { tail "$OUT/bench_$c.log"; exit 4; }
  tail -1 "$OUT/bench_$c.log"
done
