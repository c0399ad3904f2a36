#!/bin/bash
# LDS-slab march (verdict r02 #1): its bit-exactness tests, a same-box A/B of
# config 5 (brick4832 default / COL48 plain / COL48 + slab), then counters of
# the slab and plain COL48 kernels (TA / TD / L1 / LDS / VALU).
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03slab; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "slab or col48" > $OUT/pytest.log 2>&1 || { echo tests fail; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2 3; do
  for v in "" "--layout 15" "--slab"; do
    timeout -k 10 200 python -u bench.py --config grid512 $v --no-cpu-baseline --steps 40 > $OUT/b.json 2> $OUT/b.err || { echo "bench $v fail"; tail -5 $OUT/b.err; exit 4; }
    python -c "import json;j=json.loads(open('$OUT/b.json').read());print('$r', '${v:-default}', j['config']['kernel'], j['ms_per_step'], j['kernel_ms_mean'], j['roofline']['frac'])"
  done
done | tee $OUT/ab.txt
[ -n "${NOPMC:-}" ] && exit 0
PMC_LIST="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
FETCH_SIZE" timeout -k 10 400 bash tools/pmc.sh slab --size 512 --frames 10 --layout 15 --slab 1 || exit 2
python tools/pmc_summary.py slab > $OUT/pmc_slab.json; cat $OUT/pmc_slab.json
PMC_LIST="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
FETCH_SIZE" timeout -k 10 400 bash tools/pmc.sh col48 --size 512 --frames 10 --layout 15 --slab 0 || exit 2
python tools/pmc_summary.py col48 > $OUT/pmc_col48.json; cat $OUT/pmc_col48.json
