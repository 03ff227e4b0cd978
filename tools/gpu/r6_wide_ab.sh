#!/bin/bash
# Round 6: 256-row vs 288-row wide tiles (3x3 fwd / dgrad of the 'wide' shape set), two interleaved passes, cold caches
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6
for pass in 1 2; do
  for lib in libdmayolo_hip_w256.so ""; do
    echo "== pass $pass lib ${lib:-default(288)}" >> gpurun_out/r6/wide_ab.log
    DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/tune_conv.py wide fwd,dgrad >> gpurun_out/r6/wide_ab.log 2>&1 || exit $?
  done
done
cat gpurun_out/r6/wide_ab.log
