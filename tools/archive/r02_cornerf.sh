# CORNERF vs CORNERH, regions schedule (4 wedges), same box: config 4 and 1080p x 128 at 128^3
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u tools/layout_sweep.py --sizes 128 --variants 14:5:1:4,15:5:1:4 --width 3840 --height 2160 --steps 256 --rounds 7 > $OUT/sweep_cf_4k.log 2>&1 || { tail $OUT/sweep_cf_4k.log; exit 4; }
tail -3 $OUT/sweep_cf_4k.log
timeout -k 10 300 python -u tools/layout_sweep.py --sizes 128 --variants 14:5:1:4,15:5:1:4 --rounds 7 > $OUT/sweep_cf_1080.log 2>&1 || { tail $OUT/sweep_cf_1080.log; exit 4; }
tail -3 $OUT/sweep_cf_1080.log
