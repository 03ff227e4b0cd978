#!/bin/bash
# Round 6: the batch-2 conv shapes (BN partial rows at small M) and the whole-model bench-shape tests
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv_bench_shapes.py tests/test_gpu_bench_shape.py tests/test_gpu_conv.py > $OUT/fix_tests.log 2>&1
rc=$?; tail -3 $OUT/fix_tests.log; exit $rc
