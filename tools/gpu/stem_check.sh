#!/bin/bash
# conv parity incl. the s2d stem shapes on the streaming 3x3 gather, then A/B of DMY_P1S_STEM on the stem shapes
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_model.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "conv or s2d" > gpurun_out/stem_tests.log 2>&1
rc=$?; tail -3 gpurun_out/stem_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|assert|Error" gpurun_out/stem_tests.log | head -20; exit $rc; }
for cfg in DMY_P1S_STEM=0 DMY_P1S_STEM=1; do
  echo "== $cfg"
  env $cfg timeout -k 10 200 python tools/gpu/tune_conv.py stem fwd 2>&1 | grep -v amdgpu.ids || exit 1
done
