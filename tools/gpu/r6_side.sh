#!/bin/bash
# Round 6: weight-grads on a side stream (functional._WgradStream) -- the GPU tests that exercise stream order
# (graphed step, determinism, DDP on RCCL, memory, optimizer, trajectory), then the DMA-1536 / yolov5s / config-5
# step A/B (DMY_WGRAD_SIDE=0 / 1, alternating, two passes)
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_model.py tests/test_gpu_determinism.py tests/test_gpu_ddp.py tests/test_gpu_memory.py tests/test_gpu_optim.py > $OUT/side_tests.log 2>&1
rc=$?; tail -3 $OUT/side_tests.log; [ $rc -ne 0 ] && exit $rc
for pass in 1 2; do
  for side in 0 1; do
    for cfg in dma-1536 v5s-640; do
      echo "== pass $pass DMY_WGRAD_SIDE=$side $cfg" >> $OUT/side_ab.log
      DMY_WGRAD_SIDE=$side timeout -k 10 300 python bench.py --config $cfg --also none --no-cpu-baseline --no-detect --steps 10 --warmup 3 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" >> $OUT/side_ab.log || exit 1
    done
  done
done
cat $OUT/side_ab.log
