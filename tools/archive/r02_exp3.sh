#!/bin/bash
# Round 2 experiment 3: Perlin gradient-table banking (0 = interleaved pair
# table, 1 = split pair table, 2 = 16 single gradients): procedural parity,
# config 2/3 timing and LDS bank-conflict counters.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"; export TMPDIR=/tmp
for v in 0 1 2; do
  lib=volumetricrenderer_amd/libvr_ptab$v.so; [ $v = 0 ] && lib=volumetricrenderer_amd/libvr.so
  VR_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "procedural" > "$OUT/pytest_ptab$v.log" 2>&1
  rc=$?; tail -1 "$OUT/pytest_ptab$v.log"; [ $rc -ne 0 ] && exit $rc
done
for v in 0 1 2; do
  lib=volumetricrenderer_amd/libvr_ptab$v.so; [ $v = 0 ] && lib=volumetricrenderer_amd/libvr.so
  for c in cloud cloud_shadow; do
    VR_LIB=$lib timeout -k 10 300 python -u bench.py --config $c --steps 20 > "$OUT/bench_ptab${v}_$c.log" 2>&1 || { tail "$OUT/bench_ptab${v}_$c.log"; exit 4; }
    python - "$OUT/bench_ptab${v}_$c.log" $v $c <<'PY'
import json,sys
j=json.loads(open(sys.argv[1]).read().strip().split("\n")[-1])
print("ptab", sys.argv[2], sys.argv[3], "ms", j["ms_per_step"], "kernel_ms", j["kernel_ms_mean"], "frac", j["roofline"]["frac"])
PY
  done
  PMC_LIST="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS" VR_LIB=$lib timeout -k 10 200 bash tools/pmc.sh ptab$v --proc --frames 5 > /dev/null || exit 5
  python tools/pmc_summary.py ptab$v > "$OUT/pmc_ptab$v.json"; python -c "import json;d=json.loads(open('$OUT/pmc_ptab$v.json').read().split(' ',1)[1]);print('ptab $v', {k:round(v) if isinstance(v,float) and v>10 else v for k,v in d.items() if k.startswith(('SQ_LDS','SQ_INSTS','valu','SQ_WAIT'))})"
done
