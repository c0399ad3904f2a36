# Config 4 (128^3 cornerh, 3840x2160x256): TA/TD busy, VMEM, L1/L2 counters of the
# shipped kernel -- what co-limits it with the VALU (cornerf)
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"; export TMPDIR=/tmp
PMC_LIST="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum
TCC_HIT_sum TCC_MISS_sum
FETCH_SIZE" timeout -k 10 400 bash tools/pmc.sh ch4kta --size 128 --width 3840 --height 2160 --steps 256 --frames 5 || exit 2
python tools/pmc_summary.py ch4kta > "$OUT/ch4kta.json"; cat "$OUT/ch4kta.json"
