#!/bin/bash
# round 4: where the spinning config-5 frame's host time goes -- HIP API
# trace + stats of the spin bench (no counters in this run)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
rm -rf gpurun_out/prof_spin
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats -d gpurun_out/prof_spin -o run --output-format csv \
    -- python3 bench.py --config grid512 --spin --steps 64 --no-cpu-baseline --no-other-configs > gpurun_out/r04_spinprof.json 2> gpurun_out/r04_spinprof.err || { tail -5 gpurun_out/r04_spinprof.err; exit 1; }
tail -c 300 gpurun_out/r04_spinprof.json; echo
f=$(find gpurun_out/prof_spin -name "run_hip_api_stats.csv" | head -1)
head -25 "$f" | cut -d, -f1-5
