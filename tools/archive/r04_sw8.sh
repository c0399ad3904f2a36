#!/bin/bash
# round 4: config 3's shadow pass built for 8 waves per SIMD (libvr_sw8.so)
# against the default (6), interleaved x3
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for rep in 1 2 3; do
  for lib in libvr.so libvr_sw8.so; do
    VR_LIB=$PWD/volumetricrenderer_amd/$lib timeout -k 10 200 python3 -u bench.py --config cloud_shadow --steps 20 --no-cpu-baseline --no-other-configs > gpurun_out/r04_sw8_$lib.$rep.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['kernel_ms_mean'])" gpurun_out/r04_sw8_$lib.$rep.json $lib
  done
done
