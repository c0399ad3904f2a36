#!/bin/bash
# round 4: split-march unit order (tile-major vs sub-block-major): parity, then
# per rank at N = 1, 2, 4, 8 (configs 5 and 4), interleaved
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --tb=short --timeout 120 --timeout-method thread \
    -k "unit_order" > gpurun_out/r04_unit_dbg.log 2>&1 || { tail -20 gpurun_out/r04_unit_dbg.log; exit 1; }
tail -1 gpurun_out/r04_unit_dbg.log
for rep in 1 2; do for o in 0 1; do
  timeout -k 10 300 python -u tools/band_scaling.py --all-ranks --opt unit_order=$o > gpurun_out/r04_unit${o}_c5_$rep.txt 2>&1 || { tail gpurun_out/r04_unit${o}_c5_$rep.txt; exit 1; }
  grep "rank-0" gpurun_out/r04_unit${o}_c5_$rep.txt | grep -v "N=1:"
done; done
for o in 0 1; do
  timeout -k 10 300 python -u tools/band_scaling.py --all-ranks --opt unit_order=$o --size 128 --width 3840 --height 2160 --steps 256 > gpurun_out/r04_unit${o}_c4.txt 2>&1 || { tail gpurun_out/r04_unit${o}_c4.txt; exit 1; }
  grep "rank-0" gpurun_out/r04_unit${o}_c4.txt | grep -v "N=1:"
done
