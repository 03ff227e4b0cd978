#!/bin/bash
# Round-4 targeted GPU tests + a calibration micro.  Each step has its own time limit.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
TAG=${TAG:-t}
( while sleep 50; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 1000 python -u -m pytest ${T} -v -s -p no:cacheprovider --timeout 600 --timeout-method thread \
    > gpurun_out/r4/tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r4/tests_$TAG.log | tail -2; grep -E "^FAILED|^ERROR" gpurun_out/r4/tests_$TAG.log | head
[ $rc -ge 2 ] && exit $rc
if [ -n "$MICRO" ]; then
  TUNE_COLD=1 timeout -k 10 300 python -u tools/gpu/tune_conv.py $MICRO ${MICROKINDS:-fwd,fwdnb,dgrad} > gpurun_out/r4/micro_${TAG}.log 2>&1
  echo "micro rc=$?"
fi
exit $rc
