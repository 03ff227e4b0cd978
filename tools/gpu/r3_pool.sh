#!/bin/bash
# separable max-pool backward + XCD-ordered pool grids: pool / module / model / determinism tests, config-5 step + stats
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest tests/test_gpu_pools.py tests/test_gpu_modules.py tests/test_gpu_model.py tests/test_gpu_determinism.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/pool_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/pool_tests.log; grep -E "^FAILED" gpurun_out/pool_tests.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --config c5-1920 --also none --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/r03/c5_pool_bench.json 2> gpurun_out/r03/c5_pool_bench.err
rc=$?; echo "c5 rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/r03/c5_pool_bench.err; exit $rc; }
python -c "import json; d=json.loads(open('gpurun_out/r03/c5_pool_bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('detect_p50_ms'))"
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03/stats_c5_pool -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --config c5-1920 --also none --steps 3 --warmup 2 --no-cpu-baseline --no-detect > $GRAFT_REPO_ROOT/gpurun_out/r03/stats_c5_pool.log 2>&1)
rc=$?; echo "stats rc=$rc"
exit $rc
