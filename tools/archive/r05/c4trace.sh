#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r05
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
C="--size 128 --width 3840 --height 2160 --steps 256 --frames 40 --rounds 2 --streams 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4tr8 -o run -- python -u tools/band_scaling.py --native --ns 8 --rank 1 $C > $O/c4tr8.txt 2>&1 || { cat $O/c4tr8.txt; exit 3; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4tr1 -o run -- python -u tools/band_scaling.py --native --ns 1 $C > $O/c4tr1.txt 2>&1 || { cat $O/c4tr1.txt; exit 3; }
grep "N=" $O/c4tr8.txt $O/c4tr1.txt
find $O/c4tr8 $O/c4tr1 -name "*stats*"
