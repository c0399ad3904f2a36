#!/bin/bash
# Round 2, GPU session 1: GPU tests, the shipped brick4832 kernel's counters
# at 512^3 (TA/TD busy, VMEM instructions, L1/L2, FETCH), counter list.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -5 "$OUT/pytest_gpu.log"; echo "pytest rc=$rc"
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
timeout -k 10 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1; echo "list rc=$?"
PMC_LIST="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
TCC_HIT_sum TCC_MISS_sum
FETCH_SIZE" timeout -k 10 400 bash tools/pmc.sh b4832 --size 512 --frames 10 || exit 2
python tools/pmc_summary.py b4832 > "$OUT/b4832.json"; cat "$OUT/b4832.json"
echo done
