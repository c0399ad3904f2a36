#!/bin/bash
# Round-3 final evidence in one call: the whole GPU suite, smoke(), then
# tools/archive/r03_round.sh (PMC traffic of the default kernel, bench + rocprofv3 per
# config, spinning-camera lines).
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu_final.log 2>&1 || { echo "gpu tests fail"; tail -30 $OUT/pytest_gpu_final.log; exit 1; }
tail -1 $OUT/pytest_gpu_final.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke fail"; tail -20 $OUT/smoke.log; exit 2; }
tail -2 $OUT/smoke.log
bash tools/archive/r03_round.sh
