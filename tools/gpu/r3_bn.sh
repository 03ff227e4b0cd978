#!/bin/bash
# BN streaming-kernel A/B: rows per thread-iteration (DMY_BN_UNROLL) x grid cap (DMY_BN_GRID), cold operands, one process
# per setting (the knobs are read once per process).  Output gpurun_out/bn_ab.log
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/bn_ab.log
for g in 4096 8192 2048; do
  for u in 1 2 4; do
    echo "== DMY_BN_UNROLL=$u DMY_BN_GRID=$g" >> gpurun_out/bn_ab.log
    MICRO_COLD=1 MICRO_BN_ONLY=1 DMY_BN_UNROLL=$u DMY_BN_GRID=$g timeout -k 10 120 python tools/gpu/micro_elt.py >> gpurun_out/bn_ab.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { echo "rc=$rc"; exit $rc; }
  done
done
grep -v amdgpu gpurun_out/bn_ab.log
# batch-1 detect conv shapes, GPU-side time per launch (50 launches replayed from one HIP graph), warm
TUNE_GRAPH=1 timeout -k 10 200 python tools/gpu/tune_conv.py det infer > gpurun_out/det_graph.log 2>&1
rc=$?; echo "det graph rc=$rc"; grep -v amdgpu gpurun_out/det_graph.log
exit $rc
