#!/bin/bash
# Round 6: the whole GPU suite as the driver runs it (one pytest process, -m gpu), then smoke and the default bench line
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r6
mkdir -p $OUT
start=$(date +%s)
timeout -k 10 880 python -u -m pytest tests/ -x -q -m gpu --timeout 600 --timeout-method thread --durations=30 > $OUT/full_suite.log 2>&1
rc=$?
echo "suite rc=$rc wall $(( $(date +%s) - start )) s" | tee -a $OUT/full_suite.log
tail -40 $OUT/full_suite.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench_full.json 2> $OUT/bench_full.err || { tail $OUT/bench_full.err; exit 1; }
cat $OUT/bench_full.json
