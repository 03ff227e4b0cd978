#!/bin/bash
# vectorized eval epilogue: conv / model GPU tests, bs1 shapes fwd vs infer (default, DMY_P1P_EP=1), detect p50 A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_model.py tests/test_gpu_bn_fuse.py -m gpu -x -q \
  -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/epi_tests.log 2>&1 || { tail -30 gpurun_out/epi_tests.log; exit 1; }
tail -2 gpurun_out/epi_tests.log
export TUNE_GRAPH=1
timeout -k 10 200 python -u tools/gpu/tune_conv.py det fwd,infer > gpurun_out/epi_micro.log 2>&1 || exit 1
echo "== DMY_P1P_EP=1" >> gpurun_out/epi_micro.log
DMY_P1P_EP=1 timeout -k 10 200 python -u tools/gpu/tune_conv.py det infer >> gpurun_out/epi_micro.log 2>&1 || exit 1
unset TUNE_GRAPH
for cfg in dma-1536 v5s-640; do
  for p in 0 1; do
    DMY_P1P_EP=$p timeout -k 10 120 python -u tools/gpu/detect_only.py $cfg 60 2>/dev/null | sed "s/^/p1p_ep=$p /" \
      | tee -a gpurun_out/epi_det.log || exit 1
  done
done
