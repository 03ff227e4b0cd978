#!/bin/bash
# conv_sk (small-M inference GEMM): parity tests, per-shape graph timings with / without it, bs1 detect p50 A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "small_m or fill or splitk" > gpurun_out/sk_tests.log 2>&1
rc=$?; echo "sk tests rc=$rc"; tail -3 gpurun_out/sk_tests.log; grep -E "^FAILED|Error" gpurun_out/sk_tests.log | head
[ $rc -ne 0 ] && exit $rc
for sk in 0 1; do
  DMY_SK=$sk TUNE_GRAPH=1 timeout -k 10 200 python tools/gpu/tune_conv.py det infer > gpurun_out/det_graph_sk$sk.log 2>&1
  rc=$?; echo "== DMY_SK=$sk rc=$rc"; grep -v amdgpu gpurun_out/det_graph_sk$sk.log; [ $rc -ne 0 ] && exit $rc
done
for sk in 0 1 0 1; do
  for cfg in dma-1536 v5s-640; do
    DMY_SK=$sk timeout -k 10 200 python tools/gpu/detect_only.py $cfg 60 > gpurun_out/det_sk.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -5 gpurun_out/det_sk.log; exit $rc; }
    echo "DMY_SK=$sk $(grep 'detect p50' gpurun_out/det_sk.log)"
  done
done
