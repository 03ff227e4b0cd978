#!/bin/bash
# Round 6: the one-GEMM stride-2 data-grad for 32 input channels (conv_dgrad_q2s: four classes x 32 = 128 columns on
# 256 x 128 tiles; build DMY_Q2S) -- conv parity through the variant library, the data-grad A/B on the q2s shapes, then
# the yolov5s step (its 32 <- 64 @320^2 layer), alternating, two passes
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6
mkdir -p $OUT
DMY_LIB_AB=libdmayolo_hip_q2s.so timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_conv_bench_shapes.py -k "dgrad" > $OUT/q2s_tests.log 2>&1
rc=$?; tail -3 $OUT/q2s_tests.log; [ $rc -ne 0 ] && exit $rc
for pass in 1 2; do
  for lib in "" libdmayolo_hip_q2s.so; do
    echo "== pass $pass lib ${lib:-HEAD}" >> $OUT/q2s_ab.log
    DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/tune_conv.py q2s dgrad >> $OUT/q2s_ab.log 2>&1 || exit $?
  done
done
for pass in 1 2 3; do
  for lib in "" libdmayolo_hip_q2s.so; do
    DMY_LIB_AB=$lib timeout -k 10 300 python bench.py --config v5s-640 --also none --no-cpu-baseline --no-detect 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('step pass $pass lib ${lib:-HEAD}', d['value'], d['ms_per_step'])" >> $OUT/q2s_ab.log || exit 1
  done
done
grep -v amdgpu.ids $OUT/q2s_ab.log
