# A/B of the fused producer-BN reduce on one box: bench with it off / on, twice each
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for f in 0 1; do
    DMY_FUSE_BN_REDUCE=$f timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-detect > gpurun_out/b_ab_$f.log 2>&1 || exit 1
    python -c "
import json; d=json.loads(open('gpurun_out/b_ab_$f.log').read().strip().splitlines()[-1]); print('fuse=$f round=$r dma', d['value'], d['ms_per_step'], 'v5s', d['at_640']['value'], d['at_640']['ms_per_step'])"
  done
done
