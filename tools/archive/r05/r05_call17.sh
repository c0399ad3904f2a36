#!/bin/bash
# round 5, call 17: the shadow pass through the phased density (4 / 5 waves)
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
L=volumetricrenderer_amd
for v in sp sp5; do
  VR_LIB=$L/libvr_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --tb=short --timeout 120 \
      --timeout-method thread -k "procedural or worley" > $O/c17_tests_$v.log 2>&1; rc=$?
  echo "$v: $(tail -1 $O/c17_tests_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
LIBS="$L/libvr.so $L/libvr_sp.so $L/libvr_sp5.so" CONFIGS="cloud_shadow" ROUNDS=4 STEPS=30 \
    timeout -k 10 600 bash tools/abn.sh > $O/c17_ab.txt 2>&1; rc=$?
cat $O/c17_ab.txt; exit $rc
