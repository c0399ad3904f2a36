#!/bin/bash
# Round 6, call 33: config 5's region order under two frames in flight with the
# automatic 4 wedges per XCD (region_order 2, the default, against 0 and 1),
# three interleaved rounds: the gated GPU time per frame.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c33
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for round in 1 2 3; do
for ro in 2 0 1; do
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-other-configs --opt region_order=$ro \
    > $O/v.json 2> $O/v.err; rc=$?
[ $rc -eq 0 ] || { tail $O/v.err; exit $rc; }
python3 -c "
import json;d=json.loads(open('$O/v.json').read().strip().splitlines()[-1]);ro=d['roofline']
print('round $round region_order $ro:', d['ms_per_step'], ro['gpu_ms_per_frame_gated'], ro['frac_measured'])"
done
done
