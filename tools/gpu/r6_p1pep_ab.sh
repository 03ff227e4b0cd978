#!/bin/bash
# Round 6: the persistent 1x1 GEMM (conv_p1p) for inference-epilogue launches too (build DMY_P1PEP=1) against HEAD,
# graph-replayed inference launches of the bs1 @1536 layers, two interleaved passes; then the detect p50 of both
# the detect p50 of both builds
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6
mkdir -p $OUT
for pass in 1 2; do
  for lib in "" libdmayolo_hip_p1pep.so; do
    echo "== pass $pass lib ${lib:-HEAD}" >> $OUT/p1pep_ab.log
    TUNE_GRAPH=1 DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/tune_conv.py det infer >> $OUT/p1pep_ab.log 2>&1 || exit $?
    DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/detect_only.py dma-1536 60 >> $OUT/p1pep_ab.log 2>&1 || exit $?
    DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/detect_only.py v5s-640 60 >> $OUT/p1pep_ab.log 2>&1 || exit $?
  done
done
cat $OUT/p1pep_ab.log
