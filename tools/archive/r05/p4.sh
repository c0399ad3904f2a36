#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_distributed.py \
    tests/test_gpu_parity.py -k "proc or distributed or flight or spinning or sequence" > $O/p4_tests.log 2>&1 || { tail -40 $O/p4_tests.log; exit 3; }
tail -1 $O/p4_tests.log
for c in cloud cloud_shadow grid512; do
timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-other-configs > $O/p4_$c.json 2> $O/p4_$c.err || { tail -20 $O/p4_$c.err; exit 3; }
python -c "
import json,sys;d=json.loads(open('$O/p4_$c.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$c',d['value'],d['ms_per_step'],d['config']['parallelism'],r['frac'],d.get('kernel_ms_mean'))"
done
