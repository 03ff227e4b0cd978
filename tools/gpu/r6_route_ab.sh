#!/bin/bash
# Round 6: 1x1 routing A/Bs, cold caches, two interleaved passes: forward streaming GEMM limited to <= 2 column groups
# (fg2: 256 -> 768 / 1024 on the half-tile pipeline instead) and the persistent 1x1 GEMM limited to <= 128 columns
# (pm128: the 256-column views on the half-tile pipeline), against HEAD
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6
mkdir -p $OUT
for pass in 1 2; do
  for lib in "" libdmayolo_hip_fg2.so libdmayolo_hip_pm128.so; do
    echo "== pass $pass lib ${lib:-HEAD}" >> $OUT/route_ab.log
    DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/tune_conv.py p1dma fwd,dgrad >> $OUT/route_ab.log 2>&1 || exit $?
    DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/tune_conv.py p1 fwd,dgrad >> $OUT/route_ab.log 2>&1 || exit $?
  done
done
cat $OUT/route_ab.log
