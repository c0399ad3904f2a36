#!/bin/bash
# Round 6, call 12: the bench line with the gated roofline pass, plain and
# under the driver-command kernel trace.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c12
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err; rc=$?
tail -c 200 $O/bench.json; [ $rc -eq 0 ] || { tail $O/bench.err; exit $rc; }
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/drv -o bench -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/drv_bench.json 2> $O/drv_bench.err; rc=$?
[ $rc -eq 0 ] || { tail $O/drv_bench.err; exit $rc; }
