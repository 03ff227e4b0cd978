#!/bin/bash
# Round 6: conv / model / bench-shape GPU tests on HEAD, then two default DMA-1536 bench lines (no CPU baseline)
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_conv_bench_shapes.py tests/test_gpu_bench_shape.py tests/test_gpu_model.py tests/test_gpu_determinism.py tests/test_gpu_scconv_bench.py > $OUT/check_tests.log 2>&1
rc=$?; tail -3 $OUT/check_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --config dma-1536 --also v5s-640 --no-cpu-baseline --no-detect 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('check', d['value'], d['ms_per_step'], d['at_640']['value'])" >> $OUT/check_bench.log || exit 1
done
cat $OUT/check_bench.log
