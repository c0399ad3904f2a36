#!/bin/bash
# LDS bank conflicts and VALU per kernel: config 3 deferred (primary march,
# shadow pass) and the in-wave compaction, config 2 (verdict r02 #4).
set -u
export TMPDIR=/tmp
L="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
PMC_LIST="$L" timeout -k 10 200 bash tools/pmc.sh defer1 --proc --shadow 8 --frames 5 --opt shadow_defer=1 || exit 2
PMC_LIST="$L" timeout -k 10 200 bash tools/pmc.sh defer0 --proc --shadow 8 --frames 5 --opt shadow_defer=0 || exit 2
PMC_LIST="$L" timeout -k 10 200 bash tools/pmc.sh cloud2 --proc --frames 5 || exit 2
python tools/pmc_summary.py defer1:march_proc_defer defer1:proc_shadow_eval defer0:march cloud2:march | tr -d '\n' | sed 's/}/}\n/g' | tee gpurun_out/pmc_defer.txt
