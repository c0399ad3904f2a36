#!/bin/bash
# Round-end evidence: HBM traffic and L1 lookups of the default bench config
# (PMC, separate passes), then bench lines + rocprofv3 kernel-trace summaries per config.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
export TMPDIR=/tmp
PMC_LIST="FETCH_SIZE
WRITE_SIZE
TCP_TOTAL_CACHE_ACCESSES_sum TA_TA_BUSY_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD" bash tools/pmc.sh traffic512 --size 512 --frames 20 || exit 9
python tools/traffic_json.py traffic512 grid512 profiles/traffic.json || exit 9
CONFIGS="${CONFIGS:-grid512 grid128 grid4k cloud cloud_shadow}" bash tools/proc_prof.sh || exit 9
