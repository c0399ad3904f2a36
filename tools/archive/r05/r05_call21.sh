#!/bin/bash
# round 5, call 21: VALU / wait counters of the procedural kernels after the phased density
set -o pipefail
cd "$(dirname "$0")/../../.."
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
PMC_LIST="$C" timeout -k 10 300 bash tools/pmc.sh r05b_cloud --proc --frames 10 && \
PMC_LIST="$C" timeout -k 10 300 bash tools/pmc.sh r05b_cloud_shadow --proc --shadow 8 --frames 10
