#!/bin/bash
# Round 6: the one-GEMM 64-channel stride-2 data-grad (conv_dgrad_q2) -- conv parity (unit + bench shapes), then the
# s2dma data-grad A/B against the four-class launch (build DMY_Q2=0), then the p1s data-grad routing A/B
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_conv_bench_shapes.py > $OUT/q2_tests.log 2>&1
rc=$?; tail -3 $OUT/q2_tests.log; [ $rc -ne 0 ] && exit $rc
for pass in 1 2; do
  for lib in "" libdmayolo_hip_q2off.so; do
    echo "== pass $pass lib ${lib:-default(q2)}" >> $OUT/q2_ab.log
    DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/tune_conv.py s2dma dgrad >> $OUT/q2_ab.log 2>&1 || exit $?
  done
done
cat $OUT/q2_ab.log
bash tools/gpu/r6_p1sdg.sh
