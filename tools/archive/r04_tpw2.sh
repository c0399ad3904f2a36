#!/bin/bash
# round 4: smoke(), then tiles per wave x wedges x supertile around the new
# defaults (3 tiles per wave on col48, 8 wedges), config 5, interleaved x3
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r04_smoke.log 2>&1 || { tail -20 gpurun_out/r04_smoke.log; exit 1; }
tail -2 gpurun_out/r04_smoke.log
V="-1:0:0,-1:4:0,-1:3:0:16,-1:4:0:16,-1:2:0:8"
V="$V,$V,$V"
timeout -k 10 400 python -u tools/band_scaling.py --ns 1 --frames 40 --variants="$V" > gpurun_out/r04_tpw2_c5.txt 2>&1 || { tail gpurun_out/r04_tpw2_c5.txt; exit 1; }
grep "rank-0" gpurun_out/r04_tpw2_c5.txt
for st in 1 4; do
  timeout -k 10 300 python -u tools/band_scaling.py --ns 1 --frames 40 --opt supertile=$st --variants="-1:0:0,-1:0:0,-1:0:0" > gpurun_out/r04_tpw2_st$st.txt 2>&1 || exit 1
  grep "rank-0" gpurun_out/r04_tpw2_st$st.txt
done
