#!/bin/bash
# Round 6: split-K for the batch-1 k > 1 forwards up to 65536 rows (build DMY_SKM=65536) against HEAD (16384),
# graph-replayed inference launches of the bs1 @1536 layers, two interleaved passes; then the detect p50 of both
# the detect p50 of both builds
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6
mkdir -p $OUT
for pass in 1 2; do
  for lib in "" libdmayolo_hip_skm.so; do
    echo "== pass $pass lib ${lib:-HEAD}" >> $OUT/skm_ab.log
    TUNE_GRAPH=1 DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/tune_conv.py det infer >> $OUT/skm_ab.log 2>&1 || exit $?
    DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/detect_only.py dma-1536 60 >> $OUT/skm_ab.log 2>&1 || exit $?
    DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/detect_only.py v5s-640 60 >> $OUT/skm_ab.log 2>&1 || exit $?
  done
done
cat $OUT/skm_ab.log
