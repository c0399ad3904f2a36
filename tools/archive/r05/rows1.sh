#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "row_ranges" \
    tests/test_gpu_distributed.py > $O/rows_tests.log 2>&1 || { tail -40 $O/rows_tests.log; exit 3; }
tail -3 $O/rows_tests.log
for part in rows bands; do
  echo "== c4 partition $part"
  timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 2,4,8 --streams 2 --size 128 --width 3840 --height 2160 \
      --steps 256 --frames 40 --rounds 3 --partition $part > $O/rows_c4.txt 2>&1 || { cat $O/rows_c4.txt; exit 3; }
  grep -v amdgpu.ids $O/rows_c4.txt | grep -A1 "N="
done
