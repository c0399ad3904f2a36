#!/bin/bash
# Round 6, call 16: config 5's regions-schedule knobs under 2 frames in flight
# (tiles per wave, wedges per XCD, supertile), two interleaved rounds, the gated
# GPU time per frame and the host window.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/${CALL:-c16}
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for round in 1 2 3 4; do
for v in "3 8 2" "3 4 2" "3 2 2" "3 4 4" "3 8 4"; do
set -- $v
timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-other-configs \
    --opt tiles_per_wave=$1 --opt wedges=$2 --opt supertile=$3 > $O/v.json 2> $O/v.err; rc=$?
[ $rc -eq 0 ] || { tail $O/v.err; exit $rc; }
python3 -c "
import json;d=json.loads(open('$O/v.json').read().strip().splitlines()[-1]);ro=d['roofline']
print('round $round tpw $1 wedges $2 supertile $3:', d['ms_per_step'], ro['gpu_ms_per_frame_gated'], ro['frac_measured'])"
done
done
