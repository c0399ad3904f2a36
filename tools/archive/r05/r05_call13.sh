#!/bin/bash
# round 5, call 13: VALU counters of the procedural kernels (configs 2 and 3),
# each pass its own rocprofv3 run with counters only
set -o pipefail
cd "$(dirname "$0")/../../.."
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
PMC_LIST="$C" timeout -k 10 300 bash tools/pmc.sh r05_cloud --proc --frames 10 && \
PMC_LIST="$C" timeout -k 10 300 bash tools/pmc.sh r05_cloud_shadow --proc --shadow 8 --frames 10 && \
python3 tools/pmc_summary.py r05_cloud:march_proc_sorted r05_cloud_shadow:march_proc_defer r05_cloud_shadow:proc_shadow_eval \
    > gpurun_out/r05/c13_pmc.txt && cat gpurun_out/r05/c13_pmc.txt
