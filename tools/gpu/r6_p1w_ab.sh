#!/bin/bash
# Round 6: 1x1 views whose 256-row grid ends in a partial round on the 288-row wide tile (build DMY_P1W288=1) against
# the half-tile pipeline (HEAD), cold caches, two interleaved passes
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6
mkdir -p $OUT
for pass in 1 2; do
  for lib in "" libdmayolo_hip_p1w288.so; do
    echo "== pass $pass lib ${lib:-HEAD}" >> $OUT/p1w288_ab.log
    DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/tune_conv.py wide fwd,dgrad >> $OUT/p1w288_ab.log 2>&1 || exit $?
    DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/tune_conv.py p1dma fwd,dgrad >> $OUT/p1w288_ab.log 2>&1 || exit $?
  done
done
cat $OUT/p1w288_ab.log
