STEPS=tests bash tools/gpu_check.sh && for c in cloud cloud_shadow; do timeout -k 10 300 python bench.py --config $c --steps 10 --no-cpu-baseline > gpurun_out/b_${c}.log 2>&1 || exit 9; done; grep -ho "\"kernel\": \"[a-z_]*\"\|kernel_ms_mean\": [0-9.]*\|\"frac\": [0-9.]*" gpurun_out/b_*.log && PMC_LIST="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY
VALUBusy VALUUtilization" bash tools/pmc.sh cloud --proc --frames 5 && PMC_LIST="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY
VALUBusy VALUUtilization" bash tools/pmc.sh cloud_shadow --proc --shadow 8 --frames 3
