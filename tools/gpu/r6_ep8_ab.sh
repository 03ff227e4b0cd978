#!/bin/bash
# Round 6: inference 1x1 views with <= 2 K steps on the 256 x 128 tiles instead of the half-tile pipeline (build
# DMY_EP8=0) against HEAD, graph-replayed bs1 @1536 layers, two interleaved passes; then the detect p50 of both
# the detect p50 of both builds
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6
mkdir -p $OUT
for pass in 1 2; do
  for lib in "" libdmayolo_hip_ep8.so; do
    echo "== pass $pass lib ${lib:-HEAD}" >> $OUT/ep8_ab.log
    TUNE_GRAPH=1 DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/tune_conv.py det infer >> $OUT/ep8_ab.log 2>&1 || exit $?
    DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/detect_only.py dma-1536 60 >> $OUT/ep8_ab.log 2>&1 || exit $?
    DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/detect_only.py v5s-640 60 >> $OUT/ep8_ab.log 2>&1 || exit $?
  done
done
cat $OUT/ep8_ab.log
