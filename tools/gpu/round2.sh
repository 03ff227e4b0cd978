#!/bin/bash
# GPU session: full -m gpu suite, smoke, default bench (DMA-1536 headline + v5s-640), and a 2-rank gloo rehearsal of
# bench --gpus 2 on the one GPU.  Every GPU step has its own time limit; the script stops at the first failure.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-10}
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ${TESTK:+-k "$TESTK"} > gpurun_out/tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/tests.log | tail -5
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/tests.log | head -30; exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 900 python bench.py --steps $STEPS --warmup ${WARMUP:-3} ${BENCHARGS} > gpurun_out/bench.log 2>gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench.log; tail -5 gpurun_out/bench.err
if [ $rc -ne 0 ]; then exit $rc; fi
[ -n "$NODDP" ] && exit 0
timeout -k 10 300 python bench.py --gpus 2 --backend gloo --config v5s-640 --also none --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_g2.log 2>gpurun_out/bench_g2.err
rc=$?; echo "bench gloo x2 rc=$rc"; tail -c 1500 gpurun_out/bench_g2.log; tail -5 gpurun_out/bench_g2.err
exit $rc
