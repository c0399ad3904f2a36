#!/bin/bash
# Round 6, call 11: config 3's deferred shadow pass grid (option shadow_blocks),
# interleaved rounds on one box.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c11
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for round in 1 2; do
for b in 0 6144 9216 18432 24576; do
timeout -k 10 200 python3 bench.py --config cloud_shadow --steps 20 --warmup 5 --no-cpu-baseline --opt shadow_blocks=$b \
    > $O/cs_$b.json 2> $O/cs_$b.err; rc=$?
[ $rc -eq 0 ] || { tail $O/cs_$b.err; exit $rc; }
python3 -c "
import json;d=json.loads(open('$O/cs_$b.json').read().strip().splitlines()[-1]);print('round $round blocks $b', d['ms_per_step'], d['kernel_ms_mean'])"
done
done
