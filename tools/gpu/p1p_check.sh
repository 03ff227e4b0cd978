#!/bin/bash
# persistent 1x1 GEMM (DMY_P1P): conv / module parity with it forced on, then cold- and warm-cache A/B on the DMA 1x1 shapes
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
DMY_P1P=${P1PMODE:-1} timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_modules.py tests/test_gpu_model.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/p1p_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/p1p_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/p1p_tests.log | head; exit $rc; }
for cold in 1 0; do
  for m in 0 1 3; do
    echo "== DMY_P1P=$m TUNE_COLD=$cold" >> gpurun_out/p1p_ab.log
    if [ $cold = 1 ]; then export TUNE_COLD=1; else unset TUNE_COLD; fi
    DMY_P1P=$m timeout -k 10 200 python tools/gpu/tune_conv.py p1dma fwd,dgrad >> gpurun_out/p1p_ab.log 2>&1 || exit 1
  done
done
cat gpurun_out/p1p_ab.log | grep -v amdgpu
