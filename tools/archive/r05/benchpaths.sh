#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --pipeline1 --no-cpu-baseline --no-other-configs > $O/bp1.json 2> $O/bp1.err || { tail $O/bp1.err; exit 2; }
tail -c 700 $O/bp1.json; echo
timeout -k 10 300 python -u bench.py --config cloud --no-cpu-baseline --no-other-configs --pipeline1 > $O/bp2.json 2> $O/bp2.err || { tail $O/bp2.err; exit 3; }
tail -c 500 $O/bp2.json; echo
timeout -k 10 300 python -u bench.py --spin --no-cpu-baseline --no-other-configs > $O/bp3.json 2> $O/bp3.err || { tail $O/bp3.err; exit 4; }
tail -c 300 $O/bp3.json
