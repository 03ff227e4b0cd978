#!/bin/bash
# Round 5: the half-tile pipelined 256 x 256 conv (DMY_W8P): bench-shape parity with it on, then cold-cache A/B of
# every wide shape (fwd, dgrad) against the 2-stage wide loop, two interleaved passes.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r5
mkdir -p $OUT
TAG=${TAG:-w8p}
( while sleep 50; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
DMY_W8P=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_conv_bench_shapes.py > $OUT/tests_$TAG.log 2>&1
rc=$?; echo "w8p bench-shape tests rc=$rc"; tail -5 $OUT/tests_$TAG.log; [ $rc -ne 0 ] && exit $rc
for pass in 1 2; do
  for m in 0 1; do
    echo "== pass $pass DMY_W8P=$m" >> $OUT/ab_$TAG.log
    DMY_W8P=$m TUNE_COLD=1 timeout -k 10 200 python tools/gpu/tune_conv.py wide fwd,dgrad >> $OUT/ab_$TAG.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "tune rc=$rc"; tail -5 $OUT/ab_$TAG.log; exit $rc; }
  done
done
cat $OUT/ab_$TAG.log
exit 0
