#!/bin/bash
# hoisted activation switch: BN / conv / model / module GPU tests, then the 1-GPU bench and the detect p50
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_model.py tests/test_gpu_bn_fuse.py \
  tests/test_gpu_modules.py tests/test_gpu_determinism.py -m gpu -x -q -p no:cacheprovider --timeout 240 \
  --timeout-method thread > gpurun_out/act_tests.log 2>&1 || { tail -30 gpurun_out/act_tests.log; exit 1; }
tail -2 gpurun_out/act_tests.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/act_bench.json 2> gpurun_out/act_bench.err || { tail -20 gpurun_out/act_bench.err; exit 1; }
cat gpurun_out/act_bench.json
