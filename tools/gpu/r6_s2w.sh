#!/bin/bash
# Round 6: stride-2 data-grad classes on the wide / tall tiles (conv_dgrad_s2_w) -- conv parity, then the s2dma
# data-grad A/B against the 256 x 128 class tiles (build DMY_S2W=0), two interleaved passes
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_conv_bench_shapes.py > $OUT/s2w288_tests.log 2>&1
rc=$?; tail -3 $OUT/s2w288_tests.log; [ $rc -ne 0 ] && exit $rc
for pass in 1 2; do
  for lib in "" libdmayolo_hip_s2w256.so; do
    echo "== pass $pass lib ${lib:-HEAD(s2w288)}" >> $OUT/s2w288_ab.log
    DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/tune_conv.py s2dma dgrad >> $OUT/s2w288_ab.log 2>&1 || exit $?
  done
done
cat $OUT/s2w288_ab.log
