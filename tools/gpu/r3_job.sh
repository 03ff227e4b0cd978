#!/bin/bash
# Round-3 multi-part GPU job: each part under its own limit; a part that faults / aborts / times out (rc >= 2
# other than pytest's 1 = failures) ends the job.  PARTS selects: p1ptest p1pab fp8 diag
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
for part in ${PARTS:-p1ptest p1pab fp8 diag}; do
  case $part in
    p1ptest)
      DMY_P1P=${P1PMODE:-1} timeout -k 10 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_modules.py tests/test_gpu_model.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/p1p_tests.log 2>&1
      rc=$?; echo "p1ptest rc=$rc"; tail -2 gpurun_out/p1p_tests.log; grep -E "^FAILED" gpurun_out/p1p_tests.log | head -20;;
    p1pab)
      : > gpurun_out/p1p_ab.log
      rc=0
      for cold in 1 0; do
        for m in 0 1 3; do
          echo "== DMY_P1P=$m TUNE_COLD=$cold" >> gpurun_out/p1p_ab.log
          if [ $cold = 1 ]; then export TUNE_COLD=1; else unset TUNE_COLD; fi
          DMY_P1P=$m timeout -k 10 200 python tools/gpu/tune_conv.py p1dma fwd,dgrad >> gpurun_out/p1p_ab.log 2>&1
          rc=$?; [ $rc -ne 0 ] && break 2
        done
      done
      unset TUNE_COLD
      echo "p1pab rc=$rc"; grep -v amdgpu gpurun_out/p1p_ab.log;;
    fp8)
      timeout -k 10 500 python -u -m pytest tests/test_gpu_fp8.py -m gpu -v -rP -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/fp8_tests.log 2>&1
      rc=$?; echo "fp8 rc=$rc"; grep -E "passed|failed" gpurun_out/fp8_tests.log | tail -2; grep -E "^FAILED|config 5 fp8|emulation:|^jit" gpurun_out/fp8_tests.log | head -20;;
    diag)
      DIAG_ALL=0 timeout -k 10 300 python -u tools/gpu/diag_precision.py yolov5s.yaml 640 16 > gpurun_out/diag_prec_v5s_b.log 2>&1
      rc=$?; echo "diag rc=$rc"; grep -v amdgpu gpurun_out/diag_prec_v5s_b.log | head -12;;
    convtests)
      timeout -k 10 500 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_modules.py tests/test_gpu_model.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/conv_tests.log 2>&1
      rc=$?; echo "convtests rc=$rc"; tail -2 gpurun_out/conv_tests.log; grep -E "^FAILED" gpurun_out/conv_tests.log | head -20;;
    det)
      timeout -k 10 300 python tools/gpu/det_layers.py dma-1536 5 > gpurun_out/det_layers_r3.log 2>&1
      rc=$?; echo "det rc=$rc"; grep -v amdgpu gpurun_out/det_layers_r3.log | head -40;;
    c5)
      for a in "" "--fp8"; do
        timeout -k 10 400 python bench.py --config c5-1920 --also none --steps 10 --warmup 3 --no-cpu-baseline $a > gpurun_out/bench_c5${a}_r3.log 2> gpurun_out/bench_c5${a}_r3.err
        rc=$?; echo "c5 $a rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_c5${a}_r3.err; break; }
        python -c "import json,sys; d=json.loads(open('gpurun_out/bench_c5${a}_r3.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('detect_p50_ms'))"
      done;;
    bench)
      timeout -k 10 600 python bench.py --steps ${STEPS:-10} --warmup 3 ${BENCHARGS} > gpurun_out/bench_$TAG.log 2> gpurun_out/bench_$TAG.err
      rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/bench_$TAG.log;;
  esac
  ok $rc || exit $rc
done
exit 0
