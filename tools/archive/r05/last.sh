#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/last_smoke.log 2>&1 || { tail $O/last_smoke.log; exit 3; }
tail -1 $O/last_smoke.log
timeout -k 10 400 python -u bench.py > $O/last_bench.json 2> $O/last_bench.err || { tail -20 $O/last_bench.err; exit 3; }
python -c "
import json;d=json.loads(open('$O/last_bench.json').read().strip().splitlines()[-1]);r=d['roofline'];print(d['value'],d['ms_per_step'],d['config']['parallelism'],r['frac'],r.get('frac_measured'),d.get('kernel_ms_mean'));print({k:v['ms_per_step'] for k,v in d['other_configs'].items()})"
