#!/bin/bash
# Round 6: bwd1x1 tile A/B for the K = 256 column-split shapes (TP 32 default vs 64, PX 1 / 2), in-tree A/B libraries
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6
for lib in "" libdmayolo_hip_b1tp64px1.so libdmayolo_hip_b1tp64px2.so; do
  echo "== lib ${lib:-default}" >> gpurun_out/r6/b1ab.log
  DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/bwd1x1_ab.py 0 >> gpurun_out/r6/b1ab.log 2>&1 || exit $?
done
cat gpurun_out/r6/b1ab.log
