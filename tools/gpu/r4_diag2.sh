#!/bin/bash
# Round-4 diagnostics 2: trajectory (both cases) + bench-shape precision (bf16_sink emulation); p1s knob sweep;
# product-free --pmc reproduction (last: it may segfault).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
( while sleep 50; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${T:-tests/test_gpu_trajectory.py tests/test_gpu_bench_shape.py} -v -s -p no:cacheprovider \
      --timeout 600 --timeout-method thread > gpurun_out/r4/diag2_tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r4/diag2_tests.log | tail -2
  [ $rc -ge 2 ] && exit $rc
fi
if [ -n "$SWEEP" ]; then
  for cfg in "DMY_P1S=2" "DMY_P1S=2 DMY_P1S_BPC=2" "DMY_P1S=2 DMY_P1S_BPC=4 DMY_P1S_NTH=256" "DMY_P1S=2 DMY_P1S_BPC=2 DMY_P1S_NTH=1024"; do
    echo "== $cfg" >> gpurun_out/r4/sweep_p1s.log
    env $cfg TUNE_COLD=1 timeout -k 10 200 python -u tools/gpu/tune_conv.py p1s fwd,dgrad >> gpurun_out/r4/sweep_p1s.log 2>&1
    rc=$?; echo "sweep [$cfg] rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
fi
if [ -n "$MICRO" ]; then
  TUNE_COLD=1 timeout -k 10 300 python -u tools/gpu/tune_conv.py $MICRO ${MICROKINDS:-fwd,fwdnb,copy,dgrad} > gpurun_out/r4/micro2_$MICRO.log 2>&1
  rc=$?; echo "micro rc=$rc"; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$PMCREPRO" ]; then
  out=$GRAFT_REPO_ROOT/gpurun_out/r4/pmc_repro
  (cd /tmp && timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out -o run --output-format csv \
      -- python $GRAFT_REPO_ROOT/tools/gpu/${PMCREPRO_SCRIPT:-pmc_wrap_repro.py} ${PMCREPRO_ARG:-40000} > $out.log 2>&1)
  echo "pmc repro rc=$?"; tail -8 $out.log
fi
exit 0
