#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --config grid4k --no-cpu-baseline > $O/g4.json 2> $O/g4.err || { tail -20 $O/g4.err; exit 3; }
python -c "
import json;d=json.loads(open('$O/g4.json').read().strip().splitlines()[-1]);r=d['roofline'];print(d['value'],d['ms_per_step'],d['config']['parallelism'],r['frac'],d.get('kernel_ms_mean'));print(r['achieved_def'])"
