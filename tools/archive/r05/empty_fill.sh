#!/bin/bash
# empty tiles filled, not marched: the parity test, the whole GPU suite, then
# per-rank frame streams with the option on / off, and the bench line
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --tb=short --timeout 120 --timeout-method thread \
    -k "empty_tiles" > $O/ef_test.log 2>&1; rc=$?
tail -3 $O/ef_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --tb=short --timeout 120 --timeout-method thread \
    > $O/ef_suite.log 2>&1; rc=$?
tail -2 $O/ef_suite.log; [ $rc -eq 0 ] || exit $rc
for v in "" "--opt empty_fill=0"; do
  echo "== ${v:-empty_fill=1}"
  timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 1,4,8 --streams 1,2 --frames 100 --rounds 3 $v \
      > $O/ef_c5.txt 2>&1 || { cat $O/ef_c5.txt; exit 3; }
  grep -v amdgpu.ids $O/ef_c5.txt | grep -v "^native"
  timeout -k 10 300 python -u tools/band_scaling.py --native --all-ranks --ns 1,8 --streams 2 --size 128 --width 3840 \
      --height 2160 --steps 256 --frames 40 --rounds 3 $v > $O/ef_c4.txt 2>&1 || { cat $O/ef_c4.txt; exit 4; }
  grep -v amdgpu.ids $O/ef_c4.txt | grep -v "^native"
done
timeout -k 10 400 python -u bench.py --no-cpu-baseline > $O/ef_bench.json 2> $O/ef_bench.err; rc=$?
tail -c 300 $O/ef_bench.json; exit $rc
