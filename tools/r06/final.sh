#!/bin/bash
# Round 6, final evidence: the GPU suite, smoke(), the driver's bench command,
# its rocprofv3 kernel trace, the one-stream N = 1 line, and per-rank frame
# streams (config 5 bands + lead rows, config 4 row ranges) at N = 1, 2, 4, 8.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/${CALL:-final}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 120 --timeout-method thread \
    > $O/gpu_suite.log 2>&1; rc=$?
tail -2 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
tail -2 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err; rc=$?
tail -c 200 $O/bench.json; [ $rc -eq 0 ] || { tail $O/bench.err; exit $rc; }
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/drv -o bench -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_bench.json 2> $O/drv_bench.err; rc=$?
[ $rc -eq 0 ] || { tail $O/drv_bench.err; exit $rc; }
timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-other-configs --n1-loop sharder --steps 20 --warmup 5 \
    > $O/bench_n1_sharder.json 2> $O/bench_n1_sharder.err || exit 5
timeout -k 10 400 python -u tools/band_scaling.py --native --all-ranks --ns 1,2,4,8 --streams 2 --frames 100 --rounds 3 \
    > $O/native_c5.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/native_c5.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/band_scaling.py --native --all-ranks --ns 1,2,4,8 --streams 3 --size 128 --width 3840 \
    --height 2160 --steps 256 --frames 40 --rounds 3 > $O/native_c4.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/native_c4.txt; exit $rc
