set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $OUT
for r in 1 2; do
  for b in ${BLOCKS:-1536 1024 2048 3072 768}; do
    timeout -k 10 200 python -u bench.py --config cloud_shadow --opt shadow_blocks=$b --no-cpu-baseline --steps 20 > $OUT/b.json 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 4; }
    python -c "import json;j=json.loads(open('$OUT/b.json').read());print('$r blocks=$b', j['ms_per_step'], j['kernel_ms_mean'])"
  done
done | tee $OUT/ab_blocks.txt
timeout -k 10 200 python -u bench.py --config cloud_shadow --spin --steps 64 --no-cpu-baseline > $OUT/spin_cloud_shadow.json 2> $OUT/spin_cs.err || { tail -5 $OUT/spin_cs.err; exit 5; }
tail -1 $OUT/spin_cloud_shadow.json
