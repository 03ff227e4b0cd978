#!/bin/bash
# conv parity (incl. the stride-2 data-grad shapes) with the merged parity-class launch, then A/B of DMY_S2_MERGE
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
DMY_S2_MERGE=${S2TEST:-2} timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/s2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/s2_tests.log; [ $rc -ne 0 ] && { grep -E "FAILED|assert|Error" gpurun_out/s2_tests.log | head -20; exit $rc; }
for cfg in DMY_S2_MERGE=0 DMY_S2_MERGE=2; do
  echo "== $cfg"
  env $cfg timeout -k 10 200 python tools/gpu/tune_conv.py s2 dgrad 2>&1 | grep -v amdgpu.ids || exit 1
done
