#!/bin/bash
# round-2 profiles: rocprofv3 kernel stats + PMC FETCH/WRITE passes for DMA-1536 and yolov5s-640 bench steps
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in dma-1536 v5s-640; do
  ARGS="--config $cfg --also none --steps 3 --warmup 1 --no-cpu-baseline --no-detect"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/stats_$cfg -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py $ARGS > $GRAFT_REPO_ROOT/gpurun_out/stats_$cfg.log 2>&1)
  rc=$?; echo "stats $cfg rc=$rc"; [ $rc -ne 0 ] && exit $rc
  PMCTAG=$cfg PMCPASSES="fetch write" PMCTIMEOUT=300 PMCCMD="python $GRAFT_REPO_ROOT/bench.py $ARGS" bash tools/gpu/pmc.sh || exit 1
done
