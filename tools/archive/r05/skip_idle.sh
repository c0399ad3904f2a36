#!/bin/bash
# timing bound: regions launches without the idle (no estimated work) tiles
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_distributed.py -q -x --tb=short --timeout 120 \
    --timeout-method thread -k "region or split or band or loopback or solo or reference_frame or spinning" > $O/si_tests.log 2>&1; rc=$?
tail -1 $O/si_tests.log; [ $rc -eq 0 ] || exit $rc
for v in "" "VR_EXP_SKIP_IDLE=1"; do
  echo "== ${v:-default}"
  env $v timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 1,4,8 --streams 2 --frames 100 --rounds 3 \
      > $O/si_native.txt 2>&1 || { cat $O/si_native.txt; exit 3; }
  grep -v amdgpu.ids $O/si_native.txt | grep -v "^native"
  env $v timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 1,8 --streams 2 --size 128 --width 3840 \
      --height 2160 --steps 256 --frames 40 --rounds 3 > $O/si_native4.txt 2>&1 || { cat $O/si_native4.txt; exit 4; }
  grep -v amdgpu.ids $O/si_native4.txt | grep -v "^native"
done
