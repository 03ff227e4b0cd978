#!/bin/bash
# halo kernel (3x3 64 -> 64): parity tests, per-shape A/B against the implicit-GEMM tiles, bs1 detect DMY_SK A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "halo or 64-64-128 or 64-96-256" > gpurun_out/halo_tests.log 2>&1
rc=$?; echo "halo tests rc=$rc"; tail -3 gpurun_out/halo_tests.log; grep -E "^FAILED|Error" gpurun_out/halo_tests.log | head
[ $rc -ne 0 ] && exit $rc
for h in 0 1; do
  DMY_HALO=$h timeout -k 10 200 python tools/gpu/tune_conv.py halo fwd,dgrad > gpurun_out/halo_ab$h.log 2>&1
  rc=$?; echo "== DMY_HALO=$h rc=$rc"; grep -v amdgpu gpurun_out/halo_ab$h.log; [ $rc -ne 0 ] && exit $rc
done
exit 0
