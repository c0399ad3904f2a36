#!/bin/bash
# Same-box A/B timing: bench.py with libvr.so vs another build (VR_LIB),
# interleaved ROUNDS times per config (boxes of the pool differ by ~5-10 %, so
# compare builds inside one gpurun call).  Usage: LIBB=path CONFIGS="..." tools/ab.sh
# A baseline build of an earlier commit, e.g.:
#   git worktree add /tmp/base <commit> && make -C /tmp/base/volumetricrenderer_amd/csrc \
#       OUT=$PWD/volumetricrenderer_amd/libvr_base.so OBJDIR=/tmp/base_obj $PWD/volumetricrenderer_amd/libvr_base.so
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"; export TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-3}); do
  for c in ${CONFIGS:-cloud}; do
    for lib in volumetricrenderer_amd/libvr.so $LIBB; do
      VR_LIB=$lib timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --steps ${STEPS:-40} > "$OUT/ab.log" 2> "$OUT/ab.err" || { tail "$OUT/ab.err"; exit 4; }
      python -c "import json;j=json.loads(open('$OUT/ab.log').read().strip().split(chr(10))[-1]);print('$r $c $(basename $lib)', j['ms_per_step'], j['kernel_ms_mean'], j['roofline']['frac'])"
    done
  done
done
