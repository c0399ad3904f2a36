#!/bin/bash
# round 5, call 8: the assembly kernels as one row per block (no per-element
# 64-bit division); parity of the assembly + shard tests, the solo frame
# streams per rank (configs 5 and 4, exchange on render / comm streams) and a
# kernel trace of the N=8 rank-0 loop
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_parity.py -q -x --tb=short --timeout 120 \
    --timeout-method thread -k "assembl or band or shard or rccl or loopback or solo or frame or pipeline or sharder" > $O/c8_tests.log 2>&1; rc=$?
tail -3 $O/c8_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_solo8b -o solo8 -- \
    python -u tools/band_scaling.py --native --ns 8 --streams 2 --frames 100 --rounds 2 --on-render \
    > $O/c8_prof_solo8.txt 2>&1 || { tail -20 $O/c8_prof_solo8.txt; exit 2; }
for orr in "--on-render" ""; do
  timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 1,4,8 --frames 100 --rounds 3 $orr \
      > $O/c8_native_c5${orr}.txt 2>&1 || { cat $O/c8_native_c5${orr}.txt; exit 3; }
  grep -v amdgpu.ids $O/c8_native_c5${orr}.txt
done
timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 1,8 --size 128 --width 3840 --height 2160 --steps 256 \
    --frames 40 --rounds 3 --on-render > $O/c8_native_c4_onr.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/c8_native_c4_onr.txt; exit $rc
