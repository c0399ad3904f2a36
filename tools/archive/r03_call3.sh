#!/bin/bash
# Round 3, call 3: the GPU suite (COL48 staged builder, auto layout COL48),
# grid512 bench, the layout-build time at 512^3.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu3.log 2>&1 || { echo tests fail; tail -40 $OUT/pytest_gpu3.log; exit 1; }
tail -1 $OUT/pytest_gpu3.log
for r in 1 2; do
  for v in "" "--layout 12"; do
    timeout -k 10 200 python -u bench.py --config grid512 $v --no-cpu-baseline --steps 40 > $OUT/b.json 2> $OUT/b.err || { echo "bench $v fail"; tail -5 $OUT/b.err; exit 4; }
    python -c "import json;j=json.loads(open('$OUT/b.json').read());print('$r', '${v:-default}', j['config']['kernel'], j['ms_per_step'], j['kernel_ms_mean'], j['roofline']['frac'])"
  done
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/build512 -o run --output-format csv -- python3 -c "
import sys; sys.path.insert(0,'.')
import volumetricrenderer_amd as vr, torch
r=vr.Renderer(0); r.generate_volume(vr.scaled_recipe(512)); torch.cuda.synchronize()
for l in (12, 15, 12, 15): r.set_layout_preference(l)
torch.cuda.synchronize(); print('ok')
" > $OUT/build512.log 2>&1 || { echo build prof fail; tail -5 $OUT/build512.log; exit 5; }
grep -h "k_build\|k_noise\|k_pack\|k_repack" $OUT/build512/*/run_kernel_stats.csv $OUT/build512/run_kernel_stats.csv 2>/dev/null | cut -c1-160
