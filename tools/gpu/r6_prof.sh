#!/bin/bash
# (EXTRA: more bench flags, e.g. --fp8 for the config-5 leg the default bench line nests)
# Round-6 profiles of HEAD (tools/gpu/r4_prof.sh with the round-6 output dir): per-launch roofline table + layer report, rocprofv3 kernel stats, and the PMC passes
# (FETCH_SIZE, WRITE_SIZE, MFMA-busy) on the FULL 3 + 2-step bench command.  The round-3 SIGSEGV under --pmc faulted in
# librocprofiler-sdk reading one byte past a 1 MiB host mapping (the HIP kernel-argument pool) during a dispatch
# (gpurun_out/r4/pmc_crash.log); HIP_FORCE_DEV_KERNARG=1 moves the kernel arguments to device memory (KARG=0 turns it off).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${OUTDIR:-r06}
mkdir -p $OUT
( while sleep 50; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
for cfg in ${CFGS:-dma-1536 v5s-640}; do
  ARGS="--config $cfg --also none --steps ${STEPS:-3} --warmup ${WARM:-2} --no-cpu-baseline --no-detect $EXTRA"
  if [ -z "$NOTABLE" ]; then
    timeout -k 10 400 python bench.py $ARGS --layer-report --launch-table $OUT/${cfg}_launches.csv > $OUT/${cfg}_bench.json 2> $OUT/${cfg}_layers.txt
    rc=$?; echo "bench $cfg rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/${cfg}_layers.txt; exit $rc; }
  fi
  if [ -z "$NOSTATS" ]; then
    (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/stats_$cfg -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py $ARGS > $GRAFT_REPO_ROOT/$OUT/stats_$cfg.log 2>&1)
    rc=$?; echo "stats $cfg rc=$rc"; [ $rc -ne 0 ] && exit $rc
  fi
  [ -n "$NOPMC" ] && continue
  # the counter passes run 1 + 1 steps: the profiler's packet callback reads past its ring on longer runs
  PARGS="--config $cfg --also none --steps ${PSTEPS:-1} --warmup ${PWARM:-1} --no-cpu-baseline --no-detect $EXTRA"
  for pass in ${PASSES:-fetch write mfma}; do
    case $pass in
      fetch) ctr="FETCH_SIZE";;
      write) ctr="WRITE_SIZE";;
      mfma) ctr="SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES";;
    esac
    out=$GRAFT_REPO_ROOT/$OUT/pmc_${cfg}_$pass
    SEGV=""; [ -f tools/segv/libsegv_report.so ] && SEGV=1
    (cd /tmp && export DMY_SEGV_REPORT=$SEGV HIP_FORCE_DEV_KERNARG=${KARG:-1} && timeout -s KILL 400 rocprofv3 --kernel-trace --pmc $ctr -d $out -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py $PARGS > $out.log 2>&1)
    rc=$?; echo "pmc $cfg $pass rc=$rc"; [ $rc -ne 0 ] && { grep -A12 "\[segv\]" $out.log | head -30; tail -5 $out.log; exit $rc; }
  done
done
exit 0
