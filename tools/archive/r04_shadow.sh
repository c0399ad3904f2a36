#!/bin/bash
# round 4, verdict r03 #5: config 3's shadow pass.  Frame time of the three
# proc_shadow_eval variants (option shadow_cache: 0 = every sample reads its
# Worley cube from LDS, 1 = a lane keeps the cube while its cell is unchanged,
# 2 = 8 lanes per entry), then LDS / VALU counters of each (one rocprofv3
# --pmc pass per group, never with tracing domains).
set -u
export TMPDIR=/tmp PYTHONUNBUFFERED=1
cd "$(dirname "$0")/.."
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
for c in 0 1 2; do
  timeout -k 10 200 python3 -u bench.py --config cloud_shadow --steps 20 --no-cpu-baseline --no-other-configs \
      --opt shadow_cache=$c > "$OUT/r04_shadow_c$c.json" 2> "$OUT/r04_shadow_c$c.err" || { tail -5 "$OUT/r04_shadow_c$c.err"; exit 2; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('shadow_cache', sys.argv[2], d['ms_per_step'], d.get('kernel_ms_mean'))" "$OUT/r04_shadow_c$c.json" $c
done
L="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
for c in 0 1 2; do
  PMC_LIST="$L" timeout -k 10 300 bash tools/pmc.sh sh$c --proc --shadow 8 --frames 5 --opt shadow_cache=$c || exit 3
done
python3 tools/pmc_summary.py sh0:proc_shadow_eval sh1:proc_shadow_eval sh2:proc_shadow_eval | tr -d '\n' | sed 's/}/}\n/g' | tee "$OUT/r04_shadow_pmc.txt"
