#!/bin/bash
# Round 6, call 10: per-stream deferred-shadow scratch (config 3 frames two in
# flight): the procedural tests, the GPU suite, then the bench's config 3 and
# config 2 lines (one stream and two in flight) under the driver's command.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c10
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 120 --timeout-method thread \
    -k "procedural or in_flight" > $O/proc_tests.log 2>&1; rc=$?
tail -3 $O/proc_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 120 --timeout-method thread \
    > $O/gpu_suite.log 2>&1; rc=$?
tail -3 $O/gpu_suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err; rc=$?
python3 -c "
import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('c5',d['ms_per_step'],d['roofline']['frac_measured'])
for k,v in d['other_configs'].items(): print(k,v['ms_per_step'],v.get('frames_in_flight_2',{}).get('ms_per_step'))"
[ $rc -eq 0 ] || { tail $O/bench.err; exit $rc; }
for c in cloud_shadow cloud; do
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --config $c > $O/bench_$c.json 2> $O/bench_$c.err; rc=$?
tail -c 400 $O/bench_$c.json; [ $rc -eq 0 ] || { tail $O/bench_$c.err; exit $rc; }
done
