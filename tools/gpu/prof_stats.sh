#!/bin/bash
# rocprofv3 kernel stats of a short bench run: bash tools/gpu/prof_stats.sh <config> [extra bench args]
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
cfg=$1; shift
ARGS="--config $cfg --also none --steps 3 --warmup 1 --no-cpu-baseline --no-detect $*"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/stats_$cfg -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py $ARGS > $GRAFT_REPO_ROOT/gpurun_out/stats_$cfg.log 2>&1)
rc=$?; echo "stats $cfg rc=$rc"; exit $rc
