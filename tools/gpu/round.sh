#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprof kernel trace. Stops at the first crash.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-10}
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 ${TESTK:+-k "$TESTK"} > gpurun_out/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -40 gpurun_out/tests.log
if [ $rc -gt 1 ]; then echo "pytest crashed; stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
if [ $rc -gt 1 ]; then exit $rc; fi
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 600 python bench.py --steps $STEPS --warmup 3 ${BENCHARGS} > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
if [ $rc -ne 0 ]; then exit $rc; fi
[ -n "$NOPROF" ] && exit 0
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-detect ${BENCHARGS} > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 $GRAFT_REPO_ROOT/gpurun_out/prof.log
find $GRAFT_REPO_ROOT/gpurun_out/prof -name "*stats*" | head
