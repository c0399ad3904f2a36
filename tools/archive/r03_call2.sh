#!/bin/bash
# Round 3, call 2: step-major shadow dealing A/B (cloud_shadow, cloud; base =
# the round-2 compaction), the slab / COL48 counters, the quad-dedup calibration.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03; mkdir -p $OUT; export TMPDIR=/tmp
ROUNDS=3 CONFIGS="cloud_shadow cloud" LIBB=volumetricrenderer_amd/libvr_base.so bash tools/ab.sh | tee $OUT/ab_shadow_dealing.txt
bash tools/lds_dma_calib.sh > $OUT/ldscal.txt 2>&1 || { echo calib fail; tail -5 $OUT/ldscal.txt; }
tail -16 $OUT/ldscal.txt
OUT2=$GRAFT_REPO_ROOT/gpurun_out/r03slab
PMC_LIST="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_ACTIVE_INST_LDS
FETCH_SIZE" timeout -k 10 400 bash tools/pmc.sh slab --size 512 --frames 10 --layout 15 --slab 1 || exit 2
python tools/pmc_summary.py slab > $OUT2/pmc_slab.json; cat $OUT2/pmc_slab.json
PMC_LIST="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
SQ_WAIT_ANY
FETCH_SIZE" timeout -k 10 400 bash tools/pmc.sh col48 --size 512 --frames 10 --layout 15 --slab 0 || exit 2
python tools/pmc_summary.py col48 > $OUT2/pmc_col48.json; cat $OUT2/pmc_col48.json
