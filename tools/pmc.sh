#!/bin/bash
# Counter passes over one prof_case configuration, each its own rocprofv3 run
# (never combined with tracing domains).  Usage: tools/pmc.sh TAG ARGS...
set -u
TAG=$1; shift
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/pmc_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
while read -r CNTRS; do
    [ -z "$CNTRS" ] && continue
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc $CNTRS -d "$OUT/p$i" -o run --output-format csv \
        -- python3 tools/prof_case.py "$@" > "$OUT/p$i.log" 2>&1
    rc=$?
    echo "pass $i ($CNTRS) rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done <<LIST
${PMC_LIST:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY
SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM
FETCH_SIZE
WRITE_SIZE
TCC_HIT_sum TCC_MISS_sum
TA_BUSY_avr TA_TA_BUSY_sum}
LIST
