#!/bin/bash
# Round 6: batch-1 v2 tiles -- 64 x 64 unless the 128 x 128 grid fills the chip (build DMY_BIGT=1) against HEAD
# (128 x 128 from M >= 4096), graph-replayed inference launches of the bs1 @1536 layers, two interleaved passes; then
# the detect p50 of both builds
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6
mkdir -p $OUT
for pass in 1 2; do
  for lib in "" libdmayolo_hip_bigt.so; do
    echo "== pass $pass lib ${lib:-HEAD}" >> $OUT/bigt_ab.log
    TUNE_GRAPH=1 DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/tune_conv.py det infer >> $OUT/bigt_ab.log 2>&1 || exit $?
    DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/detect_only.py dma-1536 60 >> $OUT/bigt_ab.log 2>&1 || exit $?
    DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/detect_only.py v5s-640 60 >> $OUT/bigt_ab.log 2>&1 || exit $?
  done
done
cat $OUT/bigt_ab.log
