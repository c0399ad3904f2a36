#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for rnd in 1 2; do
for v in "cloud" "cloud --n1-loop sharder" "cloud_shadow"; do
set -- $v
timeout -k 10 300 python -u bench.py --config $v --no-cpu-baseline --no-other-configs > $O/p5.json 2> $O/p5.err || { tail -20 $O/p5.err; exit 3; }
python -c "
import json,sys;d=json.loads(open('$O/p5.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$v',d['value'],d['ms_per_step'],d['config']['parallelism'],r['frac'],d.get('kernel_ms_mean'))"
done
done
