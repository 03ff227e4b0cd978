#!/bin/bash
# tests (TESTS), then DMA-1536 bench A/B over the settings in ABS ("VAR=a VAR=b ..."), ROUNDS rounds, same box
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-ab}
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/tests_$TAG.log; grep -E "^FAILED" gpurun_out/tests_$TAG.log | head -20
  [ $rc -ne 0 ] && exit $rc
fi
: > gpurun_out/ab_$TAG.log
for r in $(seq ${ROUNDS:-2}); do
  for s in $ABS; do
    env $s timeout -k 10 300 python bench.py --also none --no-cpu-baseline --no-detect --steps ${STEPS:-10} --warmup 3 > gpurun_out/ab_one.json 2> gpurun_out/ab_one.err
    rc=$?; [ $rc -ne 0 ] && { echo "$s rc=$rc"; tail -3 gpurun_out/ab_one.err; exit $rc; }
    v=$(python -c "import json; d=json.loads(open('gpurun_out/ab_one.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")
    echo "round $r $s $v" | tee -a gpurun_out/ab_$TAG.log
  done
done
exit 0
