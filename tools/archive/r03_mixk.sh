#!/bin/bash
# Mixed split (long tiles KS lanes per ray, the rest 1) for small frame shares:
# parity, then rank-0 band-set times at N = 1, 2, 4, 8 (tools/band_scaling.py)
# for configs 5 and 4, interleaved.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03mixk; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "split" > $OUT/pytest.log 2>&1 || { echo tests fail; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2; do
  for pct in 0 90 70 50 30; do
    timeout -k 10 200 python -u tools/band_scaling.py --size 512 --ns 2,4,8 --opt split_long=$pct 2>&1 | grep "N=" || exit 4
    timeout -k 10 200 python -u tools/band_scaling.py --size 128 --width 3840 --height 2160 --steps 256 --ns 4,8 --opt split_long=$pct 2>&1 | sed 's/^/4k /' | grep "N=" || exit 4
  done
done | tee $OUT/ab.txt
