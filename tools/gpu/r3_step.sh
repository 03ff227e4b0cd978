#!/bin/bash
# conv / module / model GPU tests (+ TESTS override), then the default bench (TAG names the outputs)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-step}
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_conv.py tests/test_gpu_modules.py tests/test_gpu_model.py} -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/tests_$TAG.log; grep -E "^FAILED" gpurun_out/tests_$TAG.log | head -20
[ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
[ -n "$NOBENCH" ] && exit $rc
timeout -k 10 600 python bench.py --steps ${STEPS:-10} --warmup 3 ${BENCHARGS} > gpurun_out/bench_$TAG.log 2> gpurun_out/bench_$TAG.err
brc=$?; echo "bench rc=$brc"; python -c "import json; d=json.loads(open('gpurun_out/bench_$TAG.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('detect_p50_ms'), d['at_640']['value'] if 'at_640' in d else '')"
exit $(( rc > brc ? rc : brc ))
