#!/bin/bash
# Round 6, call 15: the PMC traffic record of the shipped config-5 kernel,
# re-collected on this build (FETCH_SIZE and WRITE_SIZE in separate passes,
# then the L1-lookup / TA pass), per the HBM/rocprofv3 recipe.
set -o pipefail
cd "$(dirname "$0")/../.."
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L="FETCH_SIZE
WRITE_SIZE
TCP_TOTAL_CACHE_ACCESSES_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD"
PMC_LIST="$L" timeout -k 10 500 bash tools/pmc.sh r06c5 --size 512 --frames 20 || exit 2
python3 tools/traffic_json.py r06c5 grid512 gpurun_out/r06/traffic.json
