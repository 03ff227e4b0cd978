#!/bin/bash
# Round 5: batch-1 detect profile: p50 of the graphed forward + NMS, then a rocprofv3 kernel trace of the same loop
# (per-kernel durations and the gaps between them), for DMA-YOLO-l @1536 and yolov5s @640.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r5
mkdir -p $OUT
TAG=${TAG:-det}
for cfg in ${CFGS:-dma-1536 v5s-640}; do
  timeout -k 10 200 python tools/gpu/detect_only.py $cfg 60 >> $OUT/${TAG}_p50.log 2>&1
  rc=$?; echo "p50 $cfg rc=$rc"; tail -1 $OUT/${TAG}_p50.log; [ $rc -ne 0 ] && exit $rc
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/${TAG}_$cfg -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/gpu/detect_only.py $cfg 30 > $GRAFT_REPO_ROOT/$OUT/${TAG}_$cfg.log 2>&1)
  rc=$?; echo "trace $cfg rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
