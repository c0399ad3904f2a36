#!/bin/bash
# round 4: region_order (inside-out / longest tile first / longest block first),
# parity, then per-rank timing at N = 1, 2, 4, 8 (configs 5 and 4)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --tb=short --timeout 120 --timeout-method thread \
    -k "region_order" > gpurun_out/r04_order_dbg.log 2>&1 || { tail -20 gpurun_out/r04_order_dbg.log; exit 1; }
tail -1 gpurun_out/r04_order_dbg.log
for o in 0 1 2; do
  timeout -k 10 300 python -u tools/band_scaling.py --all-ranks --opt region_order=$o > gpurun_out/r04_order${o}_c5.txt 2>&1 || { tail gpurun_out/r04_order${o}_c5.txt; exit 1; }
  grep "rank-0" gpurun_out/r04_order${o}_c5.txt
  timeout -k 10 300 python -u tools/band_scaling.py --all-ranks --opt region_order=$o --size 128 --width 3840 --height 2160 --steps 256 > gpurun_out/r04_order${o}_c4.txt 2>&1 || { tail gpurun_out/r04_order${o}_c4.txt; exit 1; }
  grep "rank-0" gpurun_out/r04_order${o}_c4.txt
done
