#!/bin/bash
# Round 6: the rest of the GPU suite, smoke, and the default bench line
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6
TAG=suiteB TLIM=700 TESTS="tests/test_gpu_droppath.py tests/test_gpu_fp8.py tests/test_gpu_loss_nms.py tests/test_gpu_memory.py tests/test_gpu_metrics.py tests/test_gpu_mha.py tests/test_gpu_model.py tests/test_gpu_modules.py tests/test_gpu_optim.py tests/test_gpu_pools.py tests/test_gpu_scconv_bench.py tests/test_gpu_tal.py tests/test_gpu_trajectory.py" bash tools/gpu/r6_tests.sh > /dev/null || { tail -30 gpurun_out/r6/suiteB.log; exit 1; }
tail -3 gpurun_out/r6/suiteB.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6/smoke.log 2>&1 || { tail gpurun_out/r6/smoke.log; exit 1; }
tail -2 gpurun_out/r6/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r6/bench.json 2> gpurun_out/r6/bench.err || { tail gpurun_out/r6/bench.err; exit 1; }
cat gpurun_out/r6/bench.json
