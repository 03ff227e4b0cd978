#!/bin/bash
# Round-4 diagnostics: bench-shape kernel parity, trajectory parity, Adam resume; 1x1 family microbench (cold);
# last: the rocprofv3 --pmc crash reproduction with the fault reporter (a segfault ends the script).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
# progress heartbeat (every step below has its own time limit)
( while sleep 50; do echo "[hb] $(date +%T) $(ls gpurun_out/r4 | wc -l) files"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
T=${T:-tests/test_gpu_conv_bench_shapes.py tests/test_gpu_trajectory.py tests/test_gpu_optim.py}
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest $T -v -s -p no:cacheprovider --timeout 300 --timeout-method thread \
      > gpurun_out/r4/diag_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r4/diag_tests.log | tail -2
  [ $rc -ge 2 ] && exit $rc
fi
if [ -n "$MICRO" ]; then
  TUNE_COLD=1 timeout -k 10 300 python -u tools/gpu/tune_conv.py ${MICRO} fwd,dgrad,wgrad > gpurun_out/r4/micro_$MICRO.log 2>&1
  rc=$?; echo "micro rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$PMCCRASH" ]; then
  out=$GRAFT_REPO_ROOT/gpurun_out/r4/pmc_crash
  (cd /tmp && DMY_SEGV_REPORT=1 timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out -o run \
      --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --config dma-1536 --also none --steps 3 --warmup 2 \
      --no-cpu-baseline --no-detect > $out.log 2>&1)
  echo "pmc rc=$?"; grep -A40 "\[segv\]" $out.log | head -80
fi
exit 0
