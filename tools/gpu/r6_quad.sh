#!/bin/bash
# Round 6: quad tile (128 x 128 per wave, conv_fwd_q) -- conv parity on the default build (quad on the 256-row wide
# grids), then the per-shape A/B against the 128 x 64 wave tiles (q0) and quad-everywhere (q2), two interleaved passes
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_conv.py tests/test_gpu_conv_bench_shapes.py > $OUT/quad_tests.log 2>&1
rc=$?; tail -3 $OUT/quad_tests.log; [ $rc -ne 0 ] && exit $rc
for pass in 1 2; do
  for lib in libdmayolo_hip_q0.so "" libdmayolo_hip_q2.so; do
    echo "== pass $pass lib ${lib:-default(quad on 256-row grids)}" >> $OUT/quad_ab.log
    DMY_LIB_AB=$lib timeout -k 10 240 python tools/gpu/tune_conv.py quad fwd,dgrad >> $OUT/quad_ab.log 2>&1 || exit $?
  done
done
cat $OUT/quad_ab.log
