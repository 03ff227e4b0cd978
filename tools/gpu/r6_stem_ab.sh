#!/bin/bash
# Round 6: the space-to-depth stem forward (conv_p1s G3) with the next tile's gathered X prefetched (stpf: 64-column
# passes, 31 spilled VGPRs; stpf1: 32-column passes, no spills) against HEAD, cold caches, alternating, two passes
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6
mkdir -p $OUT
for pass in 1 2; do
  for lib in "" libdmayolo_hip_stpf.so libdmayolo_hip_stpf1.so; do
    echo "== pass $pass lib ${lib:-HEAD}" >> $OUT/stem_pf_ab.log
    DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/tune_conv.py stem fwd >> $OUT/stem_pf_ab.log 2>&1 || exit $?
  done
done
grep -v amdgpu.ids $OUT/stem_pf_ab.log
