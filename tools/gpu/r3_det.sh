#!/bin/bash
# Halo inference epilogue: conv / model GPU tests, then batch-1 detect p50 with the halo kernel off / on
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_model.py -m gpu -x -q -p no:cacheprovider \
  --timeout 240 --timeout-method thread > gpurun_out/det_tests.log 2>&1 || { tail -30 gpurun_out/det_tests.log; exit 1; }
tail -3 gpurun_out/det_tests.log
for cfg in dma-1536 v5s-640; do
  for h in 0 1; do
    DMY_HALO=$h timeout -k 10 120 python -u tools/gpu/detect_only.py $cfg 60 2>/dev/null | sed "s/^/halo=$h /" \
      | tee -a gpurun_out/det_ab.log || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/detprof \
  -o det -- python3 $GRAFT_REPO_ROOT/tools/gpu/detect_only.py dma-1536 30 > $GRAFT_REPO_ROOT/gpurun_out/detprof.log 2>&1
