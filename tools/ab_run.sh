# Same-box check + A/B: smoke, the GPU suite, then tools/ab.sh (libvr.so vs
# volumetricrenderer_amd/libvr_base.so) for $CONFIGS, $ROUNDS rounds.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke fail; tail -20 $OUT/smoke.log; exit 3; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo tests fail; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
ROUNDS=${ROUNDS:-3} CONFIGS="${CONFIGS:-grid512}" LIBB=volumetricrenderer_amd/libvr_base.so bash tools/ab.sh
