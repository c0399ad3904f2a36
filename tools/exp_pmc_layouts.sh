set -u
export TMPDIR=/tmp
for lay in 2 6; do
PMC_LIST="FETCH_SIZE
TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVES" timeout -k 10 300 bash tools/pmc.sh lay$lay --size 512 --frames 10 --layout $lay || exit 2
done
python tools/pmc_summary.py lay2 > gpurun_out/lay2.json; python tools/pmc_summary.py lay6 > gpurun_out/lay6.json
echo ok
