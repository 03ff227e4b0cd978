#!/bin/bash
# conv parity (incl. the 1x1 streaming GEMM shapes), then A/B of DMY_P1S over the 1x1 shape sets
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/p1s_tests.log 2>&1
rc=$?; tail -5 gpurun_out/p1s_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|assert|Error" gpurun_out/p1s_tests.log | head -20; exit $rc; }
for cfg in "DMY_P1S=0" "DMY_P1S=1" ${EXTRA}; do
  echo "== $cfg"
  env $cfg timeout -k 10 200 python tools/gpu/tune_conv.py ${SET:-p1dma} fwd,dgrad 2>&1 | grep -v amdgpu.ids || exit 1
done
