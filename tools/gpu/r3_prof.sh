#!/bin/bash
# Round-3 profiles of HEAD: per-launch roofline table + layer report, rocprofv3 kernel stats, PMC
# FETCH_SIZE / WRITE_SIZE passes, for the DMA-1536 and yolov5s-640 bench steps.  Outputs under gpurun_out/r03/.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
for cfg in ${CFGS:-dma-1536 v5s-640}; do
  ARGS="--config $cfg --also none --steps 3 --warmup 2 --no-cpu-baseline --no-detect"
  timeout -k 10 400 python bench.py $ARGS --layer-report --launch-table gpurun_out/r03/${cfg}_launches.csv > gpurun_out/r03/${cfg}_bench.json 2> gpurun_out/r03/${cfg}_layers.txt
  rc=$?; echo "bench $cfg rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03/${cfg}_layers.txt; exit $rc; }
  [ -n "$NOPROF" ] && continue
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03/stats_$cfg -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py $ARGS > $GRAFT_REPO_ROOT/gpurun_out/r03/stats_$cfg.log 2>&1)
  rc=$?; echo "stats $cfg rc=$rc"; [ $rc -ne 0 ] && exit $rc
  [ -n "$NOPMC" ] && continue
  # PMC passes on 1 + 1 steps: rocprofv3 --pmc segfaults inside the HIP runtime (dmy_bn_bwd_finalize's dispatch) a few
  # seconds into the 3 + 2-step command (profiles/r03/pmc_crash.log), the short one completes
  PARGS="--config $cfg --also none --steps 1 --warmup 1 --no-cpu-baseline --no-detect"
  for pass in fetch write; do
    ctr=$([ $pass = fetch ] && echo FETCH_SIZE || echo WRITE_SIZE)
    out=$GRAFT_REPO_ROOT/gpurun_out/r03/pmc_${cfg}_$pass
    (cd /tmp && timeout -s KILL 400 rocprofv3 --kernel-trace --pmc $ctr -d $out -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py $PARGS > $out.log 2>&1)
    rc=$?; echo "pmc $cfg $pass rc=$rc"; [ $rc -ne 0 ] && { tail -5 $out.log; exit $rc; }
  done
done
exit 0
