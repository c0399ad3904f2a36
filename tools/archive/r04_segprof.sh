#!/bin/bash
# round 4: where a 1/8 share's time goes with ray segments -- march vs
# resolve kernel durations (rocprofv3 kernel trace), and the per-rank sweep
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for v in "-1:0:0:0:0:0" "-1:0:0:0:0:8" "-1:0:0:0:0:16" "-1:0:1:0:0:0"; do
  tag=$(echo "$v" | tr ':' '_')
  rm -rf gpurun_out/prof_seg$tag
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_seg$tag -o run --output-format csv \
      -- python3 tools/band_scaling.py --ns 8 --frames 50 --variants="$v" > gpurun_out/segprof$tag.txt 2>&1 || { tail -5 gpurun_out/segprof$tag.txt; exit 1; }
  grep "rank-0" gpurun_out/segprof$tag.txt
  f=$(find gpurun_out/prof_seg$tag -name "run_kernel_stats.csv" | head -1)
  head -6 "$f" | cut -d, -f1-4 | cut -c1-150
done
V="-1:0:0:0:0:0,-1:0:0:0:0:8,-1:0:0:0:0:12,-1:0:0:0:0:16,-1:0:0:0:0:24"
timeout -k 10 400 python -u tools/band_scaling.py --all-ranks --variants="$V" > gpurun_out/r04_seg2_c5.txt 2>&1 || { tail gpurun_out/r04_seg2_c5.txt; exit 1; }
grep "rank-0" gpurun_out/r04_seg2_c5.txt
