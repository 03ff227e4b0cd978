#!/bin/bash
# Round 6: stride-2 data-grad tiles for the <= 64-channel class launch (DMY_S2T builds: 0 = 256 x 64 2-stage, 1 = 256 x 64
# 3-stage, 2 = 128 x 64 2-stage, 3 = 128 x 64 3-stage), the 's2dma' shapes, two interleaved passes, cold caches
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6
mkdir -p $OUT
for pass in 1 2; do
  for lib in "" libdmayolo_hip_s2t1.so libdmayolo_hip_s2t2.so libdmayolo_hip_s2t3.so; do
    echo "== pass $pass lib ${lib:-default(256x64x2)}" >> $OUT/s2_ab.log
    DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/tune_conv.py s2dma dgrad >> $OUT/s2_ab.log 2>&1 || exit $?
  done
done
cat $OUT/s2_ab.log
