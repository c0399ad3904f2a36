#!/bin/bash
# round 5, call 19: rank 0's assembly on a side stream (VR_SHARD_ASM_PRIO /
# VR_SHARD_ASM_CUS), per-rank frame periods at N = 8 (config 5), with the
# shard tests under the CU-masked variant
set -o pipefail
cd "$(dirname "$0")/.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
VR_SHARD_ASM_CUS=16 timeout -k 10 400 python -u -m pytest tests/test_gpu_distributed.py -q -x --tb=short --timeout 120 \
    --timeout-method thread > $O/c19_dist_cus16.log 2>&1; rc=$?
tail -1 $O/c19_dist_cus16.log; [ $rc -eq 0 ] || exit $rc
for v in "" "VR_SHARD_ASM_PRIO=1" "VR_SHARD_ASM_CUS=8" "VR_SHARD_ASM_CUS=16" "VR_SHARD_ASM_CUS=32"; do
  echo "== ${v:-default}"
  env $v timeout -k 10 200 python -u tools/band_scaling.py --native --all-ranks --ns 8 --streams 2 --frames 100 --rounds 3 \
      > $O/c19_native.txt 2>&1 || { cat $O/c19_native.txt; exit 3; }
  grep -v amdgpu.ids $O/c19_native.txt | tail -2
done
