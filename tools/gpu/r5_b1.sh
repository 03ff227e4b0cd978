#!/bin/bash
# Round 5: fused 1x1 Conv-BN-act backward (bwd1x1.hip): its GPU tests, then the cold-cache A/B against the three
# launches it replaces (accumulate off / on).  EXTRA: further steps after those (a command line, run under timeout).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r5
mkdir -p $OUT
TAG=${TAG:-b1}
( while sleep 50; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_bwd1x1.py > $OUT/tests_$TAG.log 2>&1
rc=$?; echo "bwd1x1 tests rc=$rc"; tail -12 $OUT/tests_$TAG.log; [ $rc -ne 0 ] && exit $rc
for a in 0 1; do
  timeout -k 10 300 python -u tools/gpu/bwd1x1_ab.py $a >> $OUT/ab_$TAG.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "ab rc=$rc"; tail -5 $OUT/ab_$TAG.log; exit $rc; }
done
cat $OUT/ab_$TAG.log
if [ -n "$EXTRA" ]; then
  timeout -k 10 ${ETIME:-600} bash -c "$EXTRA" > $OUT/extra_$TAG.log 2>&1
  rc=$?; echo "extra rc=$rc"; tail -30 $OUT/extra_$TAG.log; [ $rc -ne 0 ] && exit $rc
fi
exit 0
