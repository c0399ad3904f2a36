#!/bin/bash
# Round-3 evidence: tools/round_profiles.sh (PMC traffic + L1 lookups of the
# default kernel, bench + rocprofv3 stats per config), then spinning-camera
# bench lines for configs 5 and 2.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/round_profiles.sh || exit 9
cp profiles/traffic.json $OUT/traffic.json
for c in grid512 cloud; do
  timeout -k 10 200 python -u bench.py --config $c --spin --steps 64 --no-cpu-baseline > $OUT/spin_$c.json 2> $OUT/spin_$c.err || { echo "spin $c fail"; tail -5 $OUT/spin_$c.err; exit 4; }
  tail -1 $OUT/spin_$c.json
done
