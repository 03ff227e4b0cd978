#!/bin/bash
# store-pattern lab, then a test list, then a micro
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
TAG=${TAG:-lab}
( while sleep 50; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
if [ -n "$LAB" ]; then
  timeout -k 10 120 ./tools/gpu/$LAB > gpurun_out/r4/${LAB}_$TAG.log 2>&1
  rc=$?; echo "lab rc=$rc"; cat gpurun_out/r4/${LAB}_$TAG.log; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$T" ]; then
  timeout -k 10 1000 python -u -m pytest $T ${TK:+-k "$TK"} -v -s -p no:cacheprovider --timeout 600 --timeout-method thread \
      > gpurun_out/r4/tests_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r4/tests_$TAG.log | tail -2; grep -E "^FAILED|^ERROR" gpurun_out/r4/tests_$TAG.log | head -20
  [ $rc -ge 2 ] && exit $rc
fi
if [ -n "$MICRO" ]; then
  TUNE_COLD=1 timeout -k 10 300 python -u tools/gpu/tune_conv.py $MICRO ${MICROKINDS:-fwd,fwdnb,dgrad} > gpurun_out/r4/micro_${TAG}.log 2>&1
  echo "micro rc=$?"
  if [ -n "$MICROAB" ]; then  # the same launches with one library knob changed, e.g. MICROAB=DMY_WGRAD_W=0
    env $MICROAB TUNE_COLD=1 timeout -k 10 300 python -u tools/gpu/tune_conv.py $MICRO ${MICROKINDS:-fwd,fwdnb,dgrad} \
        > gpurun_out/r4/micro_${TAG}_ab.log 2>&1
    echo "micro ab rc=$?"
  fi
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python bench.py $BENCH > gpurun_out/r4/bench_$TAG.json 2> gpurun_out/r4/bench_$TAG.err
  brc=$?; echo "bench rc=$brc"; tail -c 1500 gpurun_out/r4/bench_$TAG.json; tail -3 gpurun_out/r4/bench_$TAG.err
fi
exit ${rc:-0}
