#!/bin/bash
# Round 6, call 2: clock/power sampling beside per-frame periods, the GPU suite
# (slab march in the default build, the timed-path pin), the driver's bench
# command with the declared pre-warm, its kernel trace, and a 2-rank rehearsal
# of the N > 1 line's frame check (gloo, both ranks on this GPU).
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c2
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 240 python -u tools/warmup_trace.py --frames 400 --json $O/warmup_trace.json > $O/warmup_trace.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/warmup_trace.txt | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 120 --timeout-method thread \
    > $O/gpu_suite.log 2>&1; rc=$?
tail -5 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; rc=$?
tail -c 300 $O/bench.json; [ $rc -eq 0 ] || { tail $O/bench.err; exit $rc; }
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/drv -o bench -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/drv_bench.json 2> $O/drv_bench.err; rc=$?
[ $rc -eq 0 ] || { tail $O/drv_bench.err; exit $rc; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29555 bench.py --gpus 2 --steps 20 --warmup 5 --sharder torch --backend gloo \
    > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err; rc=$?
cut -c1-600 $O/bench_n2_gloo.json; [ $rc -eq 0 ] || { tail $O/bench_n2_gloo.err; exit $rc; }
