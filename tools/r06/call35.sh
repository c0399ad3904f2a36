#!/bin/bash
# Round 6, call 35: config 5's 1/8 shares (serpentine bands, lead rows) against
# the regions schedule's tiles per wave and lanes per ray (split): per-rank
# frame streams at N = 1, 8.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c35
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for v in "def:" "tpw2:--opt tiles_per_wave=2" "tpw1:--opt tiles_per_wave=1" "split1:--opt split=1" "split2:--opt split=2" "split4:--opt split=4"; do
name=${v%%:*}; args=${v#*:}
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 1,8 --streams 2 --frames 100 --rounds 3 $args \
    > $O/c5_$name.txt 2>&1; rc=$?
echo "config 5 $name"; grep -A1 "N=[18] render" $O/c5_$name.txt | grep -v "^--"; [ $rc -eq 0 ] || exit $rc
done
