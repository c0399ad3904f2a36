#!/bin/bash
# Round 3 GPU check: smoke, the GPU suite, then static and spinning-camera
# benches (grid512 = config 5, cloud = config 2, cloud_shadow = config 3).
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke fail; tail -20 $OUT/smoke.log; exit 3; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo tests fail; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for c in ${CONFIGS:-grid512 cloud cloud_shadow}; do
  for spin in "" "--spin"; do
    n=$c${spin:+_spin}
    timeout -k 10 300 python -u bench.py --config $c $spin --no-cpu-baseline --steps ${STEPS:-64} > $OUT/bench_$n.json 2> $OUT/bench_$n.err || { echo "bench $n fail"; tail -5 $OUT/bench_$n.err; exit 4; }
    python -c "import json;j=json.loads(open('$OUT/bench_$n.json').read());print('$n', j['ms_per_step'], j['kernel_ms_mean'], j.get('host_ms_per_frame'), j['roofline']['frac'], j['roofline'].get('worley_cells_per_eval'), j['roofline'].get('frac_27cell'))"
  done
done
if [ -n "${AB:-}" ]; then
  ROUNDS=${ROUNDS:-3} CONFIGS="$AB" LIBB=volumetricrenderer_amd/libvr_base.so bash tools/ab.sh | tee $OUT/ab.txt
fi
