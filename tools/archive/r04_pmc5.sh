#!/bin/bash
# round 4, verdict r03 #3: the binding unit of the shipped config-5 kernel
# (grid_col48_clamp_uG: 4 waves per SIMD) beside the same kernel built for 5
# waves per SIMD (VR_UM_ATTR, libvr_5w.so) and with every channel loaded.
# One rocprofv3 --pmc pass per counter group (never with tracing domains).
set -u
export TMPDIR=/tmp
cd "$(dirname "$0")/.."
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
G2="TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE"
G3="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"
G4="FETCH_SIZE GRBM_GUI_ACTIVE"
G5="SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_WAVE_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
LIST="$G1
$G2
$G3
$G4
$G5"
PMC_LIST="$LIST" timeout -k 10 400 bash tools/pmc.sh c5uG --size 512 --frames 5 || exit 2
PMC_LIST="$LIST" VR_LIB=$PWD/volumetricrenderer_amd/libvr_5w.so timeout -k 10 400 bash tools/pmc.sh c5uG5w --size 512 --frames 5 || exit 2
PMC_LIST="$LIST" timeout -k 10 400 bash tools/pmc.sh c5all --size 512 --frames 5 --opt uniform_skip=0 || exit 2
python tools/pmc_summary.py c5uG:march c5uG5w:march c5all:march | tr -d '\n' | sed 's/}/}\n/g' | tee gpurun_out/r04_pmc5.txt
