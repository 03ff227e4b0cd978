#!/bin/bash
# Round-3 GPU session: full -m gpu suite (no -x: every failure listed; -rP keeps the tests' printed measurements),
# smoke, default bench.  Each GPU step has its own time limit; a hang / abort ends the script.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r3}
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -v -rP -p no:cacheprovider --timeout 300 --timeout-method thread ${TESTK:+-k "$TESTK"} > gpurun_out/tests_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/tests_$TAG.log | tail -3
  grep -E "^FAILED|^ERROR" gpurun_out/tests_$TAG.log | head -30
  if [ $rc -ge 2 ] && [ $rc -ne 1 ]; then exit $rc; fi
  [ -n "$NOSMOKE" ] || { timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1; src=$?; echo "smoke rc=$src"; tail -2 gpurun_out/smoke_$TAG.log; [ $src -eq 0 ] || exit $src; }
fi
[ -n "$NOBENCH" ] && exit ${rc:-0}
timeout -k 10 900 python bench.py --steps ${STEPS:-10} --warmup ${WARMUP:-3} ${BENCHARGS} > gpurun_out/bench_$TAG.log 2>gpurun_out/bench_$TAG.err
brc=$?; echo "bench rc=$brc"; tail -c 3000 gpurun_out/bench_$TAG.log; tail -5 gpurun_out/bench_$TAG.err
exit $(( ${rc:-0} > brc ? ${rc:-0} : brc ))
