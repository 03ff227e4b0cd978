#!/bin/bash
# Round 6: the whole step, HEAD against the library at 70dc39f (before the stride-2 wide-tile classes, the batch-1
# tile rule and the inference 1x1 rule), alternating in one box, two passes
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6
mkdir -p $OUT
for pass in 1 2; do
  for lib in "" libdmayolo_hip_pre.so; do
    DMY_LIB_AB=$lib timeout -k 10 300 python bench.py --config dma-1536 --also v5s-640 --no-cpu-baseline --no-detect 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('pass $pass lib ${lib:-HEAD}', d['value'], d['ms_per_step'], d['at_640']['value'], d['at_640']['ms_per_step'])" >> $OUT/prevhead_ab.log || exit 1
  done
done
cat $OUT/prevhead_ab.log
