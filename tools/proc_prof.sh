#!/bin/bash
# Bench lines + rocprofv3 kernel-trace summaries for the procedural configs
# (2/3) and the 4K grid config (4).  Each GPU step under its own limit.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in ${CONFIGS:-cloud cloud_shadow grid4k}; do
    timeout -k 10 300 python bench.py --config $c --steps ${BSTEPS:-10} --cpu-budget 8 > "$OUT/bench_$c.log" 2>&1 || { echo "bench $c failed"; tail -5 "$OUT/bench_$c.log"; exit 9; }
    tail -1 "$OUT/bench_$c.log"
    rm -rf "$OUT/prof_$c"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$c" -o run --output-format csv \
        -- python3 bench.py --config $c --steps ${BSTEPS:-10} --no-cpu-baseline > "$OUT/prof_$c.log" 2>&1 || { echo "prof $c failed"; tail -5 "$OUT/prof_$c.log"; exit 9; }
done
echo proc_prof done
