#!/bin/bash
# Round 5: persistent stride-2 data-grad (DMY_S2P): conv parity (incl. accumulate, odd sizes) and every bench-shape
# conv, then a cold-cache A/B of the stride-2 data-grads against the one-tile kernels, two interleaved passes.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r5
mkdir -p $OUT
TAG=${TAG:-s2p}
( while sleep 50; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_conv.py tests/test_gpu_conv_bench_shapes.py > $OUT/tests_$TAG.log 2>&1
rc=$?; echo "conv tests rc=$rc"; tail -5 $OUT/tests_$TAG.log; [ $rc -ne 0 ] && exit $rc
for pass in 1 2; do
  for m in 0 1; do
    echo "== pass $pass DMY_S2P=$m" >> $OUT/ab_$TAG.log
    DMY_S2P=$m TUNE_COLD=1 timeout -k 10 200 python tools/gpu/tune_conv.py s2dma dgrad >> $OUT/ab_$TAG.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "tune rc=$rc"; tail -5 $OUT/ab_$TAG.log; exit $rc; }
  done
done
cat $OUT/ab_$TAG.log
exit 0
