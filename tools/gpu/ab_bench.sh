#!/bin/bash
# A/B of whole bench steps under env settings, all on one box: CFGS="A=1 A=2,B=3" BENCHARGS="--config dma-1536 ..."
cd $GRAFT_REPO_ROOT
for rep in ${REPS:-1}; do
for cfg in ${CFGS:-X=0}; do
  echo "== $cfg (rep $rep)"
  env $(echo $cfg | tr ',' ' ') timeout -k 10 400 python bench.py ${BENCHARGS:---steps 10 --warmup 3 --no-cpu-baseline --no-detect --also none} 2>/dev/null | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' | head -2 | tr '\n' ' '; echo
done
done
