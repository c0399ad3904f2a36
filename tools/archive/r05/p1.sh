#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > $O/p1_default.json 2> $O/p1_default.err || { tail -20 $O/p1_default.err; exit 3; }
timeout -k 10 300 python -u bench.py --pipeline1 > $O/p1_pipe.json 2> $O/p1_pipe.err || { tail -20 $O/p1_pipe.err; exit 3; }
timeout -k 10 300 python -u bench.py --pipeline1 --steps 100 > $O/p1_pipe100.json 2> $O/p1_pipe100.err || { tail -20 $O/p1_pipe100.err; exit 3; }
timeout -k 10 300 python -u bench.py --pipeline1 --config 2 > $O/p1_pipe_c2.json 2> $O/p1_pipe_c2.err || { tail -20 $O/p1_pipe_c2.err; exit 3; }
for f in p1_default p1_pipe p1_pipe100 p1_pipe_c2; do python -c "
import json,sys;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$f',d['value'],d['ms_per_step'],d['config']['parallelism'],r['frac'],r.get('frac_measured'),d.get('kernel_ms_mean'))"; done
