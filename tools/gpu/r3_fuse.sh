#!/bin/bash
# window-attention prologue + in-launch split-K combine: GPU tests, detect p50 with the combine off / on
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
DMY_SPLITK_FUSED=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_modules.py tests/test_gpu_mha.py tests/test_gpu_model.py \
  -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/fuse_tests.log 2>&1 || { tail -30 gpurun_out/fuse_tests.log; exit 1; }
tail -1 gpurun_out/fuse_tests.log
for r in 1 2; do
for cfg in dma-1536 v5s-640; do
  for f in 0 1; do
    DMY_SPLITK_FUSED=$f timeout -k 10 120 python -u tools/gpu/detect_only.py $cfg 60 2>/dev/null | sed "s/^/fused=$f /" \
      | tee -a gpurun_out/fuse_det.log || exit 1
  done
done
done
