# vr_shard_share_volume / distributed.share_volume on the GPU, then the whole suite
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest_share.log 2>&1 || { echo share tests fail; tail -40 $OUT/pytest_share.log; exit 1; }
tail -3 $OUT/pytest_share.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo tests fail; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
