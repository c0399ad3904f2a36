#!/bin/bash
# COL48Z (channel 3 as zpair): parity, then same-box A/B against COL48 at
# configs 5 (uniform G, the default) and the all-channels case, plus PMC.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03z; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "every_layout or uniform or split" > $OUT/pytest.log 2>&1 || { echo tests fail; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2 3; do
  for lay in 15 16; do
    timeout -k 10 200 python -u bench.py --config grid512 --layout $lay --no-cpu-baseline --steps 40 > $OUT/b.json 2> $OUT/b.err || { echo "bench $lay fail"; tail -5 $OUT/b.err; exit 4; }
    python -c "import json;j=json.loads(open('$OUT/b.json').read().strip().split(chr(10))[-1]);a=j.get('all_channels_loaded',{});print('$r', 'layout=$lay', j['config']['kernel'], j['ms_per_step'], j['kernel_ms_mean'], 'all-channels', a.get('kernel'), a.get('kernel_ms_mean'))"
  done
done | tee $OUT/ab.txt
for lay in 15 16; do
  PMC_LIST="FETCH_SIZE
TCP_TOTAL_CACHE_ACCESSES_sum TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD" timeout -k 10 200 bash tools/pmc.sh z$lay --size 512 --frames 10 --layout $lay || exit 2
  python tools/pmc_summary.py z$lay | tr -d '\n'; echo
done | tee $OUT/pmc.txt
