#!/bin/bash
# Time the march kernel across experimental library builds (build_exp/*.so,
# selected through VR_LIB) with tools/layout_sweep.py.  Each run checks every
# layout's image against the planar kernel's.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/variants
mkdir -p "$OUT"
for lib in ${LIBS:-base}; do
    if [ "$lib" = base ]; then export VR_LIB=; else export VR_LIB=$(pwd)/build_exp/libvr_$lib.so; fi
    timeout -k 10 300 python tools/layout_sweep.py --sizes ${SIZES:-512,128} --variants ${VARIANTS:-1:2:1,3:2:1,2:2:1,5:0:0,5:2:1} \
        --rounds ${ROUNDS:-3} --frames 10 > "$OUT/$lib.log" 2>&1 || { echo "$lib failed"; tail -5 "$OUT/$lib.log"; exit 9; }
    echo "== $lib"; grep median "$OUT/$lib.log"
done
