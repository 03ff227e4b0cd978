#!/bin/bash
# Several round-3 GPU parts in one call (the pool is congested): PARTS from  aug loader c5 prof
# each part under its own limit; a fault / abort / timeout (rc >= 124, 134, 139) ends the job, test failures do not
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
fatal() { [ $1 -ge 124 ]; }
for part in ${PARTS:-aug loader c5 prof}; do
  case $part in
    aug)
      timeout -k 10 300 python -u -m pytest tests/test_gpu_augment.py -m gpu -q -rP -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/aug_tests.log 2>&1
      rc=$?; echo "aug tests rc=$rc"; tail -2 gpurun_out/aug_tests.log; grep -E "^FAILED|render 32" gpurun_out/aug_tests.log | head;;
    loader)
      timeout -k 10 400 python -u tools/gpu/loader_bench.py 128 16 8 > gpurun_out/loader_bench.log 2> gpurun_out/loader_bench.err
      rc=$?; echo "loader rc=$rc"; cat gpurun_out/loader_bench.log; [ $rc -ne 0 ] && tail -5 gpurun_out/loader_bench.err;;
    c5)
      for a in "" "--fp8"; do
        timeout -k 10 400 python bench.py --config c5-1920 --also none --steps 10 --warmup 3 --no-cpu-baseline $a > gpurun_out/bench_c5${a}_r3.log 2> gpurun_out/bench_c5${a}_r3.err
        rc=$?; echo "c5 $a rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/bench_c5${a}_r3.err; break; }
        python -c "import json; d=json.loads(open('gpurun_out/bench_c5${a}_r3.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('detect_p50_ms'))"
      done;;
    prof)
      bash tools/gpu/r3_prof.sh; rc=$?;;
  esac
  fatal $rc && exit $rc
done
exit 0
