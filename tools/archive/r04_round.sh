#!/bin/bash
# round 4 evidence (one GPU): the default bench line (config 5 + configs 2, 3, 4
# under the same clock, measured copy peak) under rocprofv3 --kernel-trace
# --stats, the same command plain, the spinning-camera lines, and per-rank
# band-set timings of the strong-scaled shares.  Each GPU step has its own limit.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 400 python3 -u bench.py > "$OUT/r04_bench.json" 2> "$OUT/r04_bench.err" || { echo "bench failed"; tail -5 "$OUT/r04_bench.err"; exit 3; }
tail -c 600 "$OUT/r04_bench.json"; echo
rm -rf "$OUT/prof_r04"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_r04" -o run --output-format csv \
    -- python3 bench.py --cpu-budget 2 --cpu-budget-other 1 > "$OUT/r04_bench_prof.json" 2> "$OUT/r04_bench_prof.err" || { echo "prof failed"; tail -5 "$OUT/r04_bench_prof.err"; exit 4; }
for c in grid512 cloud cloud_shadow; do
  timeout -k 10 200 python3 -u bench.py --config $c --spin --steps 64 --no-cpu-baseline > "$OUT/r04_spin_$c.json" 2> "$OUT/r04_spin_$c.err" || { echo "spin $c failed"; tail -5 "$OUT/r04_spin_$c.err"; exit 5; }
  tail -c 400 "$OUT/r04_spin_$c.json"; echo
done
timeout -k 10 300 python3 -u tools/band_scaling.py --all-ranks > "$OUT/r04_bands_c5.txt" 2>&1 || { tail "$OUT/r04_bands_c5.txt"; exit 6; }
grep "rank-0" "$OUT/r04_bands_c5.txt"
timeout -k 10 300 python3 -u tools/band_scaling.py --all-ranks --size 128 --width 3840 --height 2160 --steps 256 > "$OUT/r04_bands_c4.txt" 2>&1 || { tail "$OUT/r04_bands_c4.txt"; exit 7; }
grep "rank-0" "$OUT/r04_bands_c4.txt"
echo round done
