#!/bin/bash
# persistent 1x1 GEMM: conv / model GPU tests, then A/B (DMY_P1_PERSIST 0/1) on the DMA and yolov5s 1x1 shapes
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_model.py tests/test_gpu_modules.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_p1.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t_p1.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/t_p1.log | head; exit $rc; }
AB_VAR=DMY_P1_PERSIST SET=p1dma KINDS=fwd,dgrad bash tools/gpu/ab_conv.sh > gpurun_out/ab_persist_dma.log 2>&1 || exit 1
cat gpurun_out/ab_persist_dma.log
AB_VAR=DMY_P1_PERSIST SET=p1 KINDS=fwd,dgrad bash tools/gpu/ab_conv.sh > gpurun_out/ab_persist_p1.log 2>&1 || exit 1
cat gpurun_out/ab_persist_p1.log
