#!/bin/bash
# Round 5: graphed detect (forward + NMS in one graph): its GPU test, p50 of the three detect forms per config, and a
# rocprofv3 kernel trace of the one-graph form.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r5
mkdir -p $OUT
TAG=${TAG:-det2}
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_model.py tests/test_gpu_modules.py tests/test_gpu_pools.py > $OUT/${TAG}_test.log 2>&1
rc=$?; echo "test rc=$rc"; tail -3 $OUT/${TAG}_test.log; [ $rc -ne 0 ] && exit $rc
for cfg in ${CFGS:-dma-1536 v5s-640}; do
  for mode in --eager --graph-fwd graph; do
    timeout -k 10 200 python tools/gpu/detect_only.py $cfg 80 $mode >> $OUT/${TAG}_p50.log 2>&1
    rc=$?; [ $rc -ne 0 ] && { tail -5 $OUT/${TAG}_p50.log; exit $rc; }
  done
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/${TAG}_$cfg -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/gpu/detect_only.py $cfg 30 > $GRAFT_REPO_ROOT/$OUT/${TAG}_$cfg.log 2>&1)
  rc=$?; echo "trace $cfg rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
grep detect $OUT/${TAG}_p50.log
exit 0
