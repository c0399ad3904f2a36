#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/p3_default.json 2> $O/p3_default.err || { tail -20 $O/p3_default.err; exit 3; }
timeout -k 10 300 python -u bench.py --config cloud --no-cpu-baseline > $O/p3_cloud.json 2> $O/p3_cloud.err || { tail -20 $O/p3_cloud.err; exit 3; }
timeout -k 10 300 python -u bench.py --config cloud_shadow --no-cpu-baseline > $O/p3_cloud_shadow.json 2> $O/p3_cloud_shadow.err || { tail -20 $O/p3_cloud_shadow.err; exit 3; }
timeout -k 10 300 python -u bench.py --n1-loop sharder --no-cpu-baseline --no-other-configs > $O/p3_sharder.json 2> $O/p3_sharder.err || { tail -20 $O/p3_sharder.err; exit 3; }
for f in p3_default p3_cloud p3_cloud_shadow p3_sharder; do python -c "
import json,sys;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$f',d['value'],d['ms_per_step'],d['config']['parallelism'],r['frac'],d.get('kernel_ms_mean'), d.get('all_channels_loaded',{}).get('ms_per_step'), {k:(v['ms_per_step'], v.get('frames_in_flight_2',{}).get('ms_per_step')) for k,v in d.get('other_configs',{}).items()})"; done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_distributed.py > $O/p3_dist.log 2>&1 || { tail -30 $O/p3_dist.log; exit 3; }
tail -1 $O/p3_dist.log
