#!/bin/bash
# Config 3 shadow dealing x enumeration A/B (one box, interleaved), then LDS
# bank conflicts per LDS instruction for each combination.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03deal; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "procedural or cloud or shadow or golden" > $OUT/pytest.log 2>&1 || { echo tests fail; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2 3; do
  for v in "deal=0,proc_enum=0" "deal=1,proc_enum=0" "deal=0,proc_enum=1" "deal=1,proc_enum=1"; do
    o=$(echo $v | sed 's/,/ --opt /; s/^/--opt /')
    timeout -k 10 200 python -u bench.py --config cloud_shadow $o --no-cpu-baseline --steps 20 > $OUT/b.json 2> $OUT/b.err || { echo "bench $v fail"; tail -5 $OUT/b.err; exit 4; }
    python -c "import json;j=json.loads(open('$OUT/b.json').read());print('$r', '$v', j['ms_per_step'], j['kernel_ms_mean'])"
  done
done | tee $OUT/ab.txt
for v in "0 0" "1 0" "0 1" "1 1"; do
  set -- $v
  PMC_LIST="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" timeout -k 10 200 bash tools/pmc.sh deal$1$2 --proc --shadow 8 --frames 5 --deal $1 --proc-enum $2 || exit 2
  python tools/pmc_summary.py deal$1$2 | tr -d '\n'; echo
done | tee $OUT/pmc.txt
