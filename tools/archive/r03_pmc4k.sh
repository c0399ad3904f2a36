#!/bin/bash
# Config 4 balance with the uniform-G kernel: VALU vs TA/TD (PMC, one pass each group).
set -u
export TMPDIR=/tmp
PMC_LIST="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_WAVES GRBM_GUI_ACTIVE
TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" timeout -k 10 300 bash tools/pmc.sh ch4k_uG --size 128 --width 3840 --height 2160 --steps 256 --frames 5 || exit 2
python tools/pmc_summary.py ch4k_uG
