#!/bin/bash
# Round 6: the one-launch column sum + BN finalize -- its unit tests, the BN / model / determinism / graph tests that run
# through it, then the DMA-1536 + yolov5s step against the two-launch path (DMY_FINAB=0), alternating
# (measured 13 % slower and removed with its test file tests/test_gpu_bn_finalize.py: profiles/r06/bn_colsum_finalize_ab.log)
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bn_finalize.py tests/test_gpu_determinism.py tests/test_gpu_model.py tests/test_gpu_bn_fuse.py tests/test_gpu_optim.py tests/test_gpu_config1.py > $OUT/fin_tests.log 2>&1
rc=$?; tail -3 $OUT/fin_tests.log; [ $rc -ne 0 ] && exit $rc
for pass in 1 2; do
  for ab in 0 1; do
    DMY_FINAB=$ab timeout -k 10 300 python bench.py --config dma-1536 --also v5s-640 --no-cpu-baseline --no-detect 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('step pass $pass fused $ab', d['value'], d['ms_per_step'], d['at_640']['value'], d['at_640']['ms_per_step'])" >> $OUT/fin_ab.log || exit 1
  done
done
cat $OUT/fin_ab.log
