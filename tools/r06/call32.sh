#!/bin/bash
# Round 6, call 32: the streamed shadow pass against the workgroup count of the
# shadow pass (option shadow_blocks; 0 = auto, 3/8 of the sorted waves, ~12 k
# at config 3): a wave streams more chunks with fewer workgroups, so its drain
# at the end is a smaller share.  Config 3, interleaved on one box.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c32
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for round in 1 2; do
for v in "0 0" "1 0" "1 1280" "1 2560" "1 5120" "0 1536"; do
set -- $v
timeout -k 10 200 python3 bench.py --config cloud_shadow --steps 40 --warmup 10 --no-cpu-baseline --opt shadow_stream=$1 \
    --opt shadow_blocks=$2 > $O/b.json 2> $O/b.err; rc=$?
[ $rc -eq 0 ] || { tail $O/b.err; exit $rc; }
python3 -c "
import json;d=json.loads(open('$O/b.json').read().strip().splitlines()[-1])
print('round $round shadow_stream $1 shadow_blocks $2:', d['ms_per_step'], d.get('kernel_ms_mean'))"
done
done
