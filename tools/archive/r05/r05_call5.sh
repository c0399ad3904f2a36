#!/bin/bash
# round 5, call 5: per-rank frame streams (native loop, solo rehearsal) after
# the host-cost cuts (launch cache, rank 0 in place), lanes per ray swept
# (the auto split was chosen for one stream), configs 5 and 4
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 120 ./tools/host_frame 40 > $O/c5_host_frame.txt 2>&1; rc=$?
cat $O/c5_host_frame.txt; [ $rc -eq 0 ] || exit $rc
for sp in 0 1 2 4; do
  timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 1,2,4,8 --frames 100 --rounds 3 --opt split=$sp \
      > $O/c5_native_c5_split$sp.txt 2>&1 || { cat $O/c5_native_c5_split$sp.txt; exit 2; }
  tail -8 $O/c5_native_c5_split$sp.txt
done
for sp in 0 1 2; do
  timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 1,4,8 --size 128 --width 3840 --height 2160 --steps 256 \
      --frames 40 --rounds 3 --opt split=$sp > $O/c5_native_c4_split$sp.txt 2>&1 || { cat $O/c5_native_c4_split$sp.txt; exit 3; }
  tail -6 $O/c5_native_c4_split$sp.txt
done
