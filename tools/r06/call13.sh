#!/bin/bash
# Round 6, call 13: config 5 at N = 1 with 2 / 3 / 4 render streams, interleaved rounds.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c13
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for round in 1 2 3; do
for rs in 2 3 4; do
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-other-configs --render-streams $rs \
    > $O/rs$rs.json 2> $O/rs$rs.err; rc=$?
[ $rc -eq 0 ] || { tail $O/rs$rs.err; exit $rc; }
python3 -c "
import json;d=json.loads(open('$O/rs$rs.json').read().strip().splitlines()[-1]);ro=d['roofline']
print('round $round streams $rs', d['ms_per_step'], ro['gpu_ms_per_frame_gated'], ro['frac_measured'], d['window']['gpu_window_ms'])"
done
done
# the other bench entry points still run (spinning camera, single configs)
for c in "--spin --no-other-configs" "--config grid4k" "--config grid128" "--config cloud_shadow"; do
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline $c > $O/entry.json 2> $O/entry.err; rc=$?
[ $rc -eq 0 ] || { echo "bench $c failed"; tail $O/entry.err; exit $rc; }
python3 -c "
import json;d=json.loads(open('$O/entry.json').read().strip().splitlines()[-1])
print('$c', d['ms_per_step'], d['config']['parallelism'], d.get('frame_check'), d['roofline']['frac'])"
done
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 8 --streams 2,3 --frames 100 --rounds 3 \
    > $O/c5_n8_streams.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/c5_n8_streams.txt; exit $rc
