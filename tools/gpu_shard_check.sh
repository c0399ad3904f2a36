#!/bin/bash
# GPU checks of the native multi-GPU frame loop that one GPU allows: the
# one-rank RCCL pipeline tests, bench at N=1 through the pipeline, and the
# torch/gloo sharder with 2 ranks on the one GPU.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "rccl or gloo or regions" > $OUT/pytest_shard.log 2>&1 || { echo tests fail; tail -30 $OUT/pytest_shard.log; exit 1; }
tail -2 $OUT/pytest_shard.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/b1.log 2>&1 || { echo b1 fail; tail $OUT/b1.log; exit 1; }
python -c "import json;d=json.loads(open('$OUT/b1.log').read().strip().splitlines()[-1]);print('plain    ',d['ms_per_step'],d['kernel_ms_mean'])"
timeout -k 10 300 python bench.py --no-cpu-baseline --pipeline1 > $OUT/b2.log 2>&1 || { echo b2 fail; tail $OUT/b2.log; exit 1; }
python -c "import json;d=json.loads(open('$OUT/b2.log').read().strip().splitlines()[-1]);print('pipeline1',d['ms_per_step'],d['kernel_ms_mean'],d['config']['collective'])"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --sharder torch --backend gloo --steps 10 > $OUT/b3.log 2>&1 || { echo b3 fail; tail $OUT/b3.log; exit 1; }
tail -1 $OUT/b3.log | cut -c1-300
echo ok
