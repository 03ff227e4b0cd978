#!/bin/bash
# config 5 @1920: per-layer conv timing, bf16 vs fp8 (delayed-scaling producer emit), + rocprof stats of the fp8 step
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
for a in "" "--fp8"; do
  timeout -k 10 400 python bench.py --config c5-1920 --also none --steps 3 --warmup 2 --no-cpu-baseline --no-detect --layer-report $a > gpurun_out/r03/c5${a}_bench.json 2> gpurun_out/r03/c5${a}_layers.txt
  rc=$?; echo "c5 $a rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03/c5${a}_layers.txt; exit $rc; }
done
for a in "" "--fp8"; do
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03/stats_c5$a -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --config c5-1920 --also none --steps 3 --warmup 2 --no-cpu-baseline --no-detect $a > $GRAFT_REPO_ROOT/gpurun_out/r03/stats_c5$a.log 2>&1)
  rc=$?; echo "stats c5 $a rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
