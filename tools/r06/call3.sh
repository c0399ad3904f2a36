#!/bin/bash
# Round 6, call 3: the driver's bench command with the pre-warm sized after the
# loop's set-up, and the timed window's host / GPU clock breakdown.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c3
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for i in 1 2; do
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench$i.json 2> $O/bench$i.err; rc=$?
python3 -c "
import json,sys;d=json.loads(open('$O/bench$i.json').read().strip().splitlines()[-1])
print(d['ms_per_step'],d['roofline']['frac_measured'],d['clock_warm']['frames'],d['window'],d['roofline'].get('kernel_busy_ms_per_frame'),d['frame_check'])
for k,v in d['other_configs'].items(): print(k,v['ms_per_step'],v['clock_warm']['frames'])"
[ $rc -eq 0 ] || { tail $O/bench$i.err; exit $rc; }
done
