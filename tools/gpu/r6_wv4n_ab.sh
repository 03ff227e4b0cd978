#!/bin/bash
# Round 6: weight-grads with 65..128 output channels and >= 256 GEMM columns on the 128 x 256 v4 tile (build
# DMY_WV4N=1) against the 128 x 128 v3 column tiles (HEAD), cold caches, two interleaved passes
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6
mkdir -p $OUT
timeout -k 10 300 env DMY_LIB_AB=libdmayolo_hip_wv4n.so python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_conv.py -k wgrad > $OUT/wv4n_tests.log 2>&1
rc=$?; tail -2 $OUT/wv4n_tests.log; [ $rc -ne 0 ] && exit $rc
for pass in 1 2; do
  for lib in "" libdmayolo_hip_wv4n.so; do
    echo "== pass $pass lib ${lib:-HEAD}" >> $OUT/wv4n_ab.log
    DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/tune_conv.py c128 wgrad >> $OUT/wv4n_ab.log 2>&1 || exit $?
    DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/tune_conv.py s2dma wgrad >> $OUT/wv4n_ab.log 2>&1 || exit $?
    DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/tune_conv.py p1dma wgrad >> $OUT/wv4n_ab.log 2>&1 || exit $?
  done
done
cat $OUT/wv4n_ab.log
