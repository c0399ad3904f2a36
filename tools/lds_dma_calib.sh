#!/bin/bash
# Vector-memory cost of LDS-DMA fills vs register loads (tools/lds_dma_calib.hip):
# one rocprofv3 pass per counter, one kernel-trace pass; tools/lds_dma_summary.py
# prints per-instruction figures.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/ldscal
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
for c in TCP_TOTAL_CACHE_ACCESSES_sum TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TCC_READ_REQ_sum; do
    timeout -s KILL 60 rocprofv3 --pmc $c -d "$OUT/$c" -o run --output-format csv -- ./tools/lds_dma_calib > "$OUT/$c.log" 2>&1 || { tail -3 "$OUT/$c.log"; exit 9; }
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- ./tools/lds_dma_calib > "$OUT/trace.log" 2>&1 || exit 9
python tools/lds_dma_summary.py "$OUT" | tee "$OUT/summary.txt"
