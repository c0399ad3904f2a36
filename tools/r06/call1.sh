#!/bin/bash
# Round 6, call 1: warm-up attribution (per-frame periods + clock samples from a
# cold process) and a kernel trace of the driver's exact bench command.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c1
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 240 python -u tools/warmup_trace.py --frames 400 --json $O/warmup_trace.json > $O/warmup_trace.txt 2>&1; rc=$?
cat $O/warmup_trace.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/drv -o bench -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_bench.json 2> $O/drv_bench.err; rc=$?
tail -c 600 $O/drv_bench.json; [ $rc -eq 0 ] || { tail $O/drv_bench.err; exit $rc; }
find $O/drv -name "*.csv" | head
