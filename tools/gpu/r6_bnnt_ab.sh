#!/bin/bash
# Round 6: non-temporal 16-B loads (nt1) / loads + stores (nt2) in the BN streaming passes against HEAD: the isolated
# passes (tools/gpu/bw_micro.py, two shapes), then the DMA-1536 step, alternating, two passes
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6
mkdir -p $OUT
for lib in "" libdmayolo_hip_nt1.so libdmayolo_hip_nt2.so; do
  echo "== lib ${lib:-HEAD}" >> $OUT/bnnt_ab.log
  DMY_LIB_AB=$lib timeout -k 10 120 python tools/gpu/bw_micro.py >> $OUT/bnnt_ab.log 2>&1 || exit $?
  DMY_LIB_AB=$lib timeout -k 10 120 python tools/gpu/bw_micro.py 294912 512 >> $OUT/bnnt_ab.log 2>&1 || exit $?
done
for pass in 1 2; do
  for lib in "" libdmayolo_hip_nt1.so libdmayolo_hip_nt2.so; do
    DMY_LIB_AB=$lib timeout -k 10 300 python bench.py --config dma-1536 --also none --no-cpu-baseline --no-detect 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('step pass $pass lib ${lib:-HEAD}', d['value'], d['ms_per_step'])" >> $OUT/bnnt_ab.log || exit 1
  done
done
grep -v amdgpu.ids $OUT/bnnt_ab.log
