#!/bin/bash
# rocprofv3 kernel-trace + stats of one bench configuration: BENCHARGS="..." (PROFNAME names the output dir)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
N=${PROFNAME:-prof}
cd /tmp && timeout -k 10 ${PROFTIMEOUT:-600} rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/$N -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-detect ${BENCHARGS} > $GRAFT_REPO_ROOT/gpurun_out/$N.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 $GRAFT_REPO_ROOT/gpurun_out/$N.log
exit $rc
