#!/bin/bash
# Round 6: 3x3 stride-1 layers with 65..128 output channels on the persistent register-epilogue GEMM (conv_p1p over the
# implicit-GEMM gather, build DMY_P3P) -- conv / BN parity through the variant library, the c128 shapes A/B, then the
# DMA-1536 + yolov5s step, alternating, two passes
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6
mkdir -p $OUT
DMY_LIB_AB=libdmayolo_hip_p3p.so timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_conv_bench_shapes.py tests/test_gpu_model.py tests/test_gpu_determinism.py > $OUT/p3p_tests.log 2>&1
rc=$?; tail -3 $OUT/p3p_tests.log; [ $rc -ne 0 ] && exit $rc
for pass in 1 2; do
  for lib in "" libdmayolo_hip_p3p.so; do
    echo "== pass $pass lib ${lib:-HEAD}" >> $OUT/p3p_ab.log
    DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/tune_conv.py c128 fwd,dgrad >> $OUT/p3p_ab.log 2>&1 || exit $?
  done
done
for pass in 1 2; do
  for lib in "" libdmayolo_hip_p3p.so; do
    DMY_LIB_AB=$lib timeout -k 10 300 python bench.py --config dma-1536 --also v5s-640 --no-cpu-baseline --no-detect 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('step pass $pass lib ${lib:-HEAD}', d['value'], d['ms_per_step'], d['at_640']['value'], d['at_640']['ms_per_step'])" >> $OUT/p3p_ab.log || exit 1
  done
done
grep -v amdgpu.ids $OUT/p3p_ab.log
