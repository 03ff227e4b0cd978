#!/bin/bash
# Round 6: window-attention backward grid size (total blocks 2048 = HEAD, 1536 = two whole rounds of 3 blocks/CU,
# 768 = one round) -- isolated kernel times (tools/gpu/swin_bench.py), then the DMA-1536 step, alternating, two passes
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6
mkdir -p $OUT
for lib in "" libdmayolo_hip_wab1536.so libdmayolo_hip_wab768.so; do
  echo "== lib ${lib:-HEAD}" >> $OUT/wab_ab.log
  DMY_LIB_AB=$lib timeout -k 10 120 python tools/gpu/swin_bench.py >> $OUT/wab_ab.log 2>&1 || exit $?
done
for pass in 1 2; do
  for lib in "" libdmayolo_hip_wab1536.so libdmayolo_hip_wab768.so; do
    DMY_LIB_AB=$lib timeout -k 10 300 python bench.py --config dma-1536 --also none --no-cpu-baseline --no-detect 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('step pass $pass lib ${lib:-HEAD}', d['value'], d['ms_per_step'])" >> $OUT/wab_ab.log || exit 1
  done
done
grep -v amdgpu.ids $OUT/wab_ab.log
