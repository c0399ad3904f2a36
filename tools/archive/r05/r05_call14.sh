#!/bin/bash
# round 5, call 14: LDS / wait counters of the procedural kernels (configs 2, 3)
set -o pipefail
cd "$(dirname "$0")/../../.."
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/r05
C="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE"
PMC_LIST="$C" timeout -k 10 300 bash tools/pmc.sh r05_cloud_lds --proc --frames 10 && \
PMC_LIST="$C" timeout -k 10 300 bash tools/pmc.sh r05_cloud_shadow_lds --proc --shadow 8 --frames 10
