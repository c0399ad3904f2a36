#!/bin/bash
# Round 2 experiment 4: procedural parity + timing + LDS counters after the
# region-ordered sort and the re-banked tables; config-4 bench vs sweep.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "procedural" > "$OUT/pytest_proc.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_proc.log"; [ $rc -ne 0 ] && exit $rc
for c in cloud cloud_shadow grid4k; do
  timeout -k 10 300 python -u bench.py --config $c --steps 40 > "$OUT/bench_$c.log" 2>&1 || { tail "$OUT/bench_$c.log"; exit 4; }
  python -c "import json,sys;j=json.loads(open('$OUT/bench_$c.log').read().strip().split(chr(10))[-1]);print('$c', j['ms_per_step'], j['kernel_ms_mean'], j['roofline']['frac'])"
done
timeout -k 10 300 python -u tools/layout_sweep.py --sizes 128 --width 3840 --height 2160 --steps 256 --variants 14:5:2:4 --rounds 5 --no-check > "$OUT/sweep_ch_4k.log" 2>&1 || exit 5
grep -v amdgpu.ids "$OUT/sweep_ch_4k.log" | head -1
PMC_LIST="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS" timeout -k 10 200 bash tools/pmc.sh proc2 --proc --frames 5 > /dev/null || exit 6
python tools/pmc_summary.py proc2 > "$OUT/pmc_proc2.json"; cat "$OUT/pmc_proc2.json"
PMC_LIST="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS" timeout -k 10 200 bash tools/pmc.sh proc3 --proc --shadow 8 --frames 3 > /dev/null || exit 7
python tools/pmc_summary.py proc3 > "$OUT/pmc_proc3.json"; cat "$OUT/pmc_proc3.json"
