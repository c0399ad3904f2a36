#!/bin/bash
# Round 6, call 36: hardware queues per process (GPU_MAX_HW_QUEUES, HIP's
# default 4) against 8: the driver's command for config 5 and the 4K rows-mode
# rehearsal whose first pipeline ran slow (c23/c24), interleaved on one box.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c36
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for round in 1 2 3; do
for q in 4 8; do
GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-other-configs --no-cpu-baseline \
    > $O/b.json 2> $O/b.err || { tail $O/b.err; exit 5; }
python3 -c "
import json;d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]);ro=d['roofline']
print('round $round queues $q:', d['ms_per_step'], 'gated', ro['gpu_ms_per_frame_gated'], 'fm', ro['frac_measured'])"
done
done
for q in 4 8; do
GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 8 --streams 3 --size 128 --width 3840 \
    --height 2160 --steps 256 --frames 40 --rounds 3 --partition rows > $O/c4_rows_q$q.txt 2>&1 || exit 6
echo "config 4 rows N=8 only, queues $q"; grep -A1 "N=8 render" $O/c4_rows_q$q.txt
done
