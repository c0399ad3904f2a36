#!/bin/bash
# Bench lines + rocprofv3 kernel-trace summaries for the procedural configs
# (2/3) and the 4K grid config (4).  Each GPU step under its own limit.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
# One run per config under the kernel trace: the bench line (with its HIP-event
# kernel mean) and the rocprof statistics come from the same process, so the
# two averages describe the same launches (runs differ by a few percent).
for c in ${CONFIGS:-cloud cloud_shadow grid4k}; do
    rm -rf "$OUT/prof_$c"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$c" -o run --output-format csv \
        -- python3 bench.py --config $c --steps ${BSTEPS:-10} --cpu-budget 8 > "$OUT/bench_$c.log" 2>&1 || { echo "bench $c failed"; tail -5 "$OUT/bench_$c.log"; exit 9; }
    grep '^{' "$OUT/bench_$c.log" | tail -1
done
echo proc_prof done
