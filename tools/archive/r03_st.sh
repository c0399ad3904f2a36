#!/bin/bash
# Supertile order of the regions list (4 waves per workgroup): same-box A/B.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03st; mkdir -p $OUT; export TMPDIR=/tmp
for r in 1 2 3 4 5; do
  for c in ${CONFIGS:-grid512 grid4k grid128}; do
    for st in 1 2 4; do
      timeout -k 10 200 python -u bench.py --config $c --opt supertile=$st --no-cpu-baseline --steps 60 > $OUT/b.json 2> $OUT/b.err || { echo "bench $c $st fail"; tail -5 $OUT/b.err; exit 4; }
      python -c "import json;j=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]);print('$r', '$c', 'st=$st', j['ms_per_step'], j['kernel_ms_mean'], j['roofline']['frac'])"
    done
  done
done | tee $OUT/ab.txt
