#!/bin/bash
# Round 6, call 38: the dealt shadow pass (option shadow_deal).  The procedural GPU
# tests, then config 3 dealt against a lane per entry, interleaved on one box, and
# the shadow pass kernel time under rocprof.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c38
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu --maxfail 5 -q --tb=short --timeout 120 --timeout-method thread \
    -k "procedural or config3 or shadow or cloud or defer" > $O/gpu_proc.log 2>&1; rc=$?
tail -3 $O/gpu_proc.log; [ $rc -eq 0 ] || exit $rc
for round in 1 2 3; do
for st in 1 0; do
timeout -k 10 200 python3 bench.py --config cloud_shadow --steps 40 --warmup 10 --no-cpu-baseline --opt shadow_deal=$st \
    > $O/b.json 2> $O/b.err; rc=$?
[ $rc -eq 0 ] || { tail $O/b.err; exit $rc; }
python3 -c "
import json;d=json.loads(open('$O/b.json').read().strip().splitlines()[-1])
print('round $round shadow_deal $st:', d['ms_per_step'], d.get('kernel_ms_mean'), d['roofline']['frac'])"
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c3 -- \
    python3 bench.py --config cloud_shadow --steps 40 --warmup 10 --no-cpu-baseline > $O/prof.json 2> $O/prof.err
