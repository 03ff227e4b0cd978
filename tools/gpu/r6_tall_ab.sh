#!/bin/bash
# Round 6: the tall 512 x 128 tile for the 65..128-column k > 1 views against the 256 x 128 3-stage tile (build
# DMY_TALL=0), cold caches, two interleaved passes (c128 3x3 shapes and the 64 -> 128 stride-2 forward)
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6
mkdir -p $OUT
for pass in 1 2; do
  for lib in "" libdmayolo_hip_notall.so; do
    echo "== pass $pass lib ${lib:-HEAD}" >> $OUT/tall_ab.log
    DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/tune_conv.py c128 fwd,dgrad >> $OUT/tall_ab.log 2>&1 || exit $?
    DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/tune_conv.py s2dma fwd >> $OUT/tall_ab.log 2>&1 || exit $?
  done
done
cat $OUT/tall_ab.log
