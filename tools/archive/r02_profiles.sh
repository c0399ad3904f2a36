#!/bin/bash
# Round 2 evidence: GPU suite, smoke, HBM traffic PMC of the default config,
# bench lines + rocprofv3 kernel stats per config, PMC of the cache-resident
# (cornerh) and procedural kernels, per-wave timeline of the 512^3 frame.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p "$OUT"; export TMPDIR=/tmp
if [ -z "${SKIP_TESTS:-}" ]; then   # SKIP_TESTS=1: suite and smoke already run in an earlier call
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -1 "$OUT/pytest_gpu.log"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail "$OUT/smoke.log"; exit 3; }
tail -1 "$OUT/smoke.log"
fi
PMC_LIST="FETCH_SIZE
WRITE_SIZE" timeout -k 10 400 bash tools/pmc.sh traffic512 --size 512 --frames 20 || exit 9
python tools/traffic_json.py traffic512 grid512 profiles/traffic.json || exit 9
CONFIGS="grid512 grid128 grid4k cloud cloud_shadow" BSTEPS=20 bash tools/proc_prof.sh || exit 9
PMC_LIST="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY" timeout -k 10 300 bash tools/pmc.sh ch4k --size 128 --width 3840 --height 2160 --steps 256 --frames 5 > /dev/null || exit 10
python tools/pmc_summary.py ch4k > "$OUT/pmc_ch4k.json"
PMC_LIST="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS" timeout -k 10 200 bash tools/pmc.sh cloud --proc --frames 5 > /dev/null || exit 11
python tools/pmc_summary.py cloud > "$OUT/pmc_cloud.json"
PMC_LIST="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS" timeout -k 10 200 bash tools/pmc.sh cloud_shadow --proc --shadow 8 --frames 3 > /dev/null || exit 12
python tools/pmc_summary.py cloud_shadow > "$OUT/pmc_cloud_shadow.json"
VR_LIB=volumetricrenderer_amd/libvr_tl.so timeout -k 10 180 python -u tools/timeline.py --json "$OUT/tl_512.json" > "$OUT/tl_512.log" 2>&1 || exit 13
echo profiles done
