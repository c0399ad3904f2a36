#!/bin/bash
# round 5, call 16: the phased density (lattice loads first, Worley cube while
# they fly) and the batched Worley cube reads: procedural parity with each
# variant library, then the A/B on configs 2 and 3
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=volumetricrenderer_amd
for v in ph pc cb; do
  VR_LIB=$L/libvr_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --tb=short --timeout 120 \
      --timeout-method thread -k "procedural or worley" > $O/c16_tests_$v.log 2>&1; rc=$?
  echo "$v: $(tail -1 $O/c16_tests_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
LIBS="$L/libvr.so $L/libvr_ph.so $L/libvr_pc.so $L/libvr_cb.so" CONFIGS="cloud cloud_shadow" ROUNDS=3 STEPS=30 \
    timeout -k 10 800 bash tools/abn.sh > $O/c16_ab.txt 2>&1; rc=$?
cat $O/c16_ab.txt; exit $rc
