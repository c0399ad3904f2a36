#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for w in 300 20; do
timeout -k 10 400 python -u bench.py --warmup $w --no-cpu-baseline > $O/wu.json 2> $O/wu.err || { tail -20 $O/wu.err; exit 3; }
python -c "
import json;d=json.loads(open('$O/wu.json').read().strip().splitlines()[-1]);r=d['roofline'];print('warmup $w',d['value'],d['ms_per_step'],r['frac'],r.get('frac_measured'),d.get('kernel_ms_mean'), {k:(v['ms_per_step'], v.get('frames_in_flight_2',{}).get('ms_per_step')) for k,v in d.get('other_configs',{}).items()})"
done
