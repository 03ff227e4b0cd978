#!/bin/bash
# Round 5: a GPU test subset (TESTS, pytest -k / paths) and optionally the default bench (driver flags).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r5
mkdir -p $OUT
TAG=${TAG:-x}
( while sleep 50; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
if [ -n "$TESTS" ]; then
  timeout -k 10 ${TTIME:-900} python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $TESTS > $OUT/tests_$TAG.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -15 $OUT/tests_$TAG.log; [ $rc -ne 0 ] && exit $rc
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 900 python bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARMUP:-5} $BENCHARGS > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
  rc=$?; echo "bench rc=$rc"; tail -c 1500 $OUT/bench_$TAG.json; [ $rc -ne 0 ] && { tail -20 $OUT/bench_$TAG.err; exit $rc; }
fi
exit 0
