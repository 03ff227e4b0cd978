#!/bin/bash
# phased wide tile (DMY_W8=1): conv / module / model / determinism GPU tests with it on, per-shape A/B, bench A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
DMY_W8=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_modules.py tests/test_gpu_model.py tests/test_gpu_determinism.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/w8_tests.log 2>&1
rc=$?; echo "w8 tests rc=$rc"; tail -2 gpurun_out/w8_tests.log; grep -E "^FAILED" gpurun_out/w8_tests.log | head -20
[ $rc -ne 0 ] && exit $rc
for m in 0 1; do
  DMY_W8=$m timeout -k 10 200 python tools/gpu/tune_conv.py dma fwd,dgrad > gpurun_out/w8_ab$m.log 2>&1
  rc=$?; echo "== DMY_W8=$m rc=$rc"; grep -v amdgpu gpurun_out/w8_ab$m.log; [ $rc -ne 0 ] && exit $rc
done
TAG=w8 ROUNDS=2 ABS="DMY_W8=0 DMY_W8=1" bash tools/gpu/r3_ab.sh
