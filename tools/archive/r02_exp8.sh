#!/bin/bash
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"; export TMPDIR=/tmp
for v in 1 2; do
  VR_LIB=volumetricrenderer_amd/libvr_key$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "procedural" > "$OUT/pytest_key$v.log" 2>&1 || { tail "$OUT/pytest_key$v.log"; exit 2; }
  tail -1 "$OUT/pytest_key$v.log"
done
for r in 1 2; do
  for c in cloud cloud_shadow; do
    for lib in volumetricrenderer_amd/libvr.so volumetricrenderer_amd/libvr_key1.so volumetricrenderer_amd/libvr_key2.so; do
      VR_LIB=$lib timeout -k 10 300 python -u bench.py --config $c --steps 40 --no-cpu-baseline > "$OUT/ab.log" 2>&1 || { tail "$OUT/ab.log"; exit 4; }
      python -c "import json;j=json.loads(open('$OUT/ab.log').read().strip().split(chr(10))[-1]);print('$r $c $(basename $lib)', j['ms_per_step'], j['kernel_ms_mean'], j['roofline']['frac'])"
    done
  done
done
for v in 1 2; do
  PMC_LIST="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU" VR_LIB=volumetricrenderer_amd/libvr_key$v.so timeout -k 10 200 bash tools/pmc.sh key$v --proc --frames 5 > /dev/null || exit 5
  python tools/pmc_summary.py key$v | tail -n +1 | tr -d '\n'; echo
done
