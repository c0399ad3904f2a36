#!/bin/bash
# round 4: spin lines (host time per frame enqueued without queue waits; the
# GPU build's code object preloaded) and the default bench line (measured copy peak)
set -o pipefail
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
export PYTHONUNBUFFERED=1
for c in grid512 cloud cloud_shadow; do
  timeout -k 10 200 python3 -u bench.py --config $c --spin --steps 64 --no-cpu-baseline > $OUT/r04_spin2_$c.json 2> $OUT/r04_spin2_$c.err || { tail -5 $OUT/r04_spin2_$c.err; exit 5; }
  python3 -c "import json; d=json.loads(open('$OUT/r04_spin2_$c.json').read().strip().splitlines()[-1]); print('$c', d['ms_per_step'], d.get('kernel_ms_mean'), d.get('host_ms_per_frame'), d.get('host_ms_per_frame_queued'), d.get('region_lists'))"
done
timeout -k 10 400 python3 -u bench.py > $OUT/r04_bench2.json 2> $OUT/r04_bench2.err || { tail -5 $OUT/r04_bench2.err; exit 3; }
python3 -c "import json; d=json.loads(open('$OUT/r04_bench2.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline'].get('peak_measured'), d['roofline'].get('frac_measured'))"
