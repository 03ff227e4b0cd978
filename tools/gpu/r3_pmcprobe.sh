#!/bin/bash
# PMC FETCH_SIZE pass on a short bench (1 + 1 steps): default kernels, then DMY_HALO=0 (which change broke --pmc?)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
ARGS="--config dma-1536 --also none --steps 1 --warmup 1 --no-cpu-baseline --no-detect"
for h in ${HALOS:-1 0}; do
  out=$GRAFT_REPO_ROOT/gpurun_out/r03/pmcprobe_h$h
  (cd /tmp && DMY_HALO=$h timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py $ARGS > $out.log 2>&1)
  rc=$?; echo "pmc halo=$h rc=$rc"; grep -E "dmy_|Abort" $out.log | head -5
  [ $rc -ne 0 ] && [ $rc -ne 139 ] && exit $rc
done
exit 0
