#!/bin/bash
# Workgroup size x supertile order of the regions schedule: parity, then a
# same-box A/B at configs 5 and 4, and L1 misses per VMEM instruction.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03wg; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "workgroups or every_layout or split" > $OUT/pytest.log 2>&1 || { echo tests fail; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2 3; do
  for c in grid512 grid4k; do
    for v in "4 1" "8 1" "16 1" "4 2" "8 2" "16 4"; do
      set -- $v
      timeout -k 10 200 python -u bench.py --config $c --opt wg_waves=$1 --opt supertile=$2 --no-cpu-baseline --steps 40 > $OUT/b.json 2> $OUT/b.err || { echo "bench $c $v fail"; tail -5 $OUT/b.err; exit 4; }
      python -c "import json;j=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]);print('$r', '$c', 'wg=$1 st=$2', j['ms_per_step'], j['kernel_ms_mean'], j['roofline']['frac'])"
    done
  done
done | tee $OUT/ab.txt
for v in "4 1" "16 1" "16 4"; do
  set -- $v
  PMC_LIST="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD" timeout -k 10 200 bash tools/pmc.sh wg$1st$2 --size 512 --frames 10 --opt wg_waves=$1 --opt supertile=$2 || exit 2
  python tools/pmc_summary.py wg$1st$2 | tr -d '\n'; echo
done | tee $OUT/pmc.txt
