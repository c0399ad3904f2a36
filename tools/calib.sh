#!/bin/bash
# L1/TA cost of gather patterns (tools/tcp_calib.hip): one rocprofv3 pass per
# counter plus one kernel-trace pass for durations.
set -u
OUT=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/calib
rm -rf "$OUT"; mkdir -p "$OUT"
export TMPDIR=/tmp
for c in TCP_TOTAL_CACHE_ACCESSES_sum TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum; do
    timeout -k 10 120 rocprofv3 --pmc $c -d "$OUT/$c" -o run --output-format csv -- ./tools/tcp_calib > "$OUT/$c.log" 2>&1 || { tail -3 "$OUT/$c.log"; exit 9; }
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- ./tools/tcp_calib > "$OUT/trace.log" 2>&1 || exit 9
echo calib done
