#!/bin/bash
# Round 6: batch-1 detect p50 (graph) and the per-kernel breakdown of one graphed detect call, DMA-1536 and yolov5s
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r6
mkdir -p $OUT
for cfg in dma-1536 v5s-640; do
  timeout -k 10 300 python tools/gpu/detect_only.py $cfg 60 >> $OUT/det_p50.log 2>&1 || exit $?
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace -d $GRAFT_REPO_ROOT/$OUT/det_$cfg -o run --output-format csv -- python $GRAFT_REPO_ROOT/tools/gpu/detect_only.py $cfg 20 > $GRAFT_REPO_ROOT/$OUT/det_$cfg.log 2>&1) || exit $?
  python tools/det_trace_summary.py $(find $OUT/det_$cfg -name '*kernel_trace.csv' | head -1) 40 > $OUT/det_${cfg}_summary.txt
done
cat $OUT/det_p50.log $OUT/det_*_summary.txt
