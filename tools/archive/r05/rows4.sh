#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_distributed.py \
    > $O/rows_dist.log 2>&1 || { tail -40 $O/rows_dist.log; exit 3; }
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "row_ranges or in_place or empty_tiles" \
    >> $O/rows_dist.log 2>&1 || { tail -40 $O/rows_dist.log; exit 3; }
grep passed $O/rows_dist.log
for part in rows bands; do
  echo "== c4 partition $part"
  timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 1,2,4,8 --streams 2 --size 128 --width 3840 --height 2160 \
      --steps 256 --frames 40 --rounds 3 --partition $part > $O/rows_c4_$part.txt 2>&1 || { cat $O/rows_c4_$part.txt; exit 3; }
  grep -v amdgpu.ids $O/rows_c4_$part.txt | grep -A1 "N="
done
