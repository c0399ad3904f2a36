#!/bin/bash
# Round 6, call 34: the roofline's gated pass behind 8 frames of the loop
# instead of a sleep kernel: the driver's command twice, the spinning camera,
# and the driver's command under rocprof for tools/trace_frames.py.
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/r06/c34
mkdir -p $O
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for k in 1 2; do
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-other-configs --no-cpu-baseline > $O/b$k.json 2> $O/b$k.err || { tail $O/b$k.err; exit 5; }
python3 -c "
import json;d=json.loads(open('$O/b$k.json').read().strip().splitlines()[-1]);ro=d['roofline']
print('run $k:', d['ms_per_step'], 'gated', ro['gpu_ms_per_frame_gated'], 'gpu window/frame', round(d['window']['gpu_window_ms']/20, 5), 'frac_measured', ro['frac_measured'], d['frame_check'])"
done
timeout -k 10 300 python3 bench.py --spin --steps 20 --warmup 5 --no-other-configs --no-cpu-baseline > $O/spin.json 2> $O/spin.err || { tail $O/spin.err; exit 6; }
tail -c 300 $O/spin.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/drv -o bench -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/drv_bench.json 2> $O/drv_bench.err || { tail $O/drv_bench.err; exit 7; }
