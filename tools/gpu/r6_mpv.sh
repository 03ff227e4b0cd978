#!/bin/bash
# Round 6: LDS max-pool tiles for k <= 5 (TH x TW pixels x CVB 16-B channel vectors per block; HEAD = 16 x 32 x 1):
# pool parity per variant library, then the isolated kernels (tools/gpu/pool_micro.py), two passes
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6
mkdir -p $OUT
for lib in libdmayolo_hip_mpv0.so libdmayolo_hip_mpv1.so libdmayolo_hip_mpv2.so libdmayolo_hip_mpv3.so; do
  DMY_LIB_AB=$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_pools.py > $OUT/mpv_tests_$lib.log 2>&1
  rc=$?; echo "$lib tests: $(tail -1 $OUT/mpv_tests_$lib.log)"; [ $rc -ne 0 ] && exit $rc
done
for pass in 1 2; do
  for lib in "" libdmayolo_hip_mpv0.so libdmayolo_hip_mpv1.so libdmayolo_hip_mpv2.so libdmayolo_hip_mpv3.so; do
    echo "== pass $pass lib ${lib:-HEAD}" >> $OUT/mpv_ab.log
    DMY_LIB_AB=$lib timeout -k 10 120 python tools/gpu/pool_micro.py >> $OUT/mpv_ab.log 2>&1 || exit $?
  done
done
grep -v amdgpu.ids $OUT/mpv_ab.log
