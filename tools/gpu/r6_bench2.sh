#!/bin/bash
# Round 6: two DMA-1536 + yolov5s bench lines (no CPU baseline, no detect)
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6
mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 300 python bench.py --config dma-1536 --also v5s-640 --no-cpu-baseline --no-detect 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('bench2', d['value'], d['ms_per_step'], d['at_640']['value'], d['at_640']['ms_per_step'])" >> $OUT/bench2.log || exit 1
done
cat $OUT/bench2.log
