#!/bin/bash
# Round 6: output-heavy 1x1 data-grads (dx channels >= 2 x dy channels) on the streaming GEMM (conv_p1s) vs the
# LDS-DMA tiles they take now (build DMY_P1SDG=1 vs default), the p1dma shapes, two interleaved passes
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6
mkdir -p $OUT
for pass in 1 2; do
  for lib in "" libdmayolo_hip_p1sdg.so; do
    echo "== pass $pass lib ${lib:-default}" >> $OUT/p1sdg_ab.log
    DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/tune_conv.py p1dma dgrad >> $OUT/p1sdg_ab.log 2>&1 || exit $?
  done
done
cat $OUT/p1sdg_ab.log
