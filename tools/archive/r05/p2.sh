#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > $O/p2_default.json 2> $O/p2_default.err || { tail -20 $O/p2_default.err; exit 3; }
timeout -k 10 300 python -u bench.py --n1-loop sharder --no-cpu-baseline --no-other-configs > $O/p2_sharder.json 2> $O/p2_sharder.err || { tail -20 $O/p2_sharder.err; exit 3; }
timeout -k 10 300 python -u bench.py --spin --no-cpu-baseline > $O/p2_spin.json 2> $O/p2_spin.err || { tail -20 $O/p2_spin.err; exit 3; }
timeout -k 10 300 python -u bench.py --config cloud --no-cpu-baseline > $O/p2_cloud.json 2> $O/p2_cloud.err || { tail -20 $O/p2_cloud.err; exit 3; }
timeout -k 10 300 python -u bench.py --config cloud_shadow --no-cpu-baseline > $O/p2_cloud_shadow.json 2> $O/p2_cloud_shadow.err || { tail -20 $O/p2_cloud_shadow.err; exit 3; }
timeout -k 10 300 python -u bench.py --config grid4k --no-cpu-baseline > $O/p2_grid4k.json 2> $O/p2_grid4k.err || { tail -20 $O/p2_grid4k.err; exit 3; }
for f in p2_default p2_sharder p2_spin p2_cloud p2_cloud_shadow p2_grid4k; do python -c "
import json,sys;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$f',d['value'],d['ms_per_step'],d['config']['parallelism'],r['frac'],d.get('kernel_ms_mean'), d.get('all_channels_loaded',{}).get('ms_per_step'), {k:(v['ms_per_step'], v.get('frames_in_flight_2',{}).get('ms_per_step')) for k,v in d.get('other_configs',{}).items()})"; done
