#!/bin/bash
# Several python runs in one GPU session: SWEEP="args1;args2;..." (each the arguments of one `python` call).
# Stops at the first failing run.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
IFS=';' read -ra RUNS <<< "$SWEEP"
for args in "${RUNS[@]}"; do
  i=$((i+1))
  echo "== run $i: $args"
  timeout -k 10 ${RUNTIMEOUT:-400} python $args > gpurun_out/sweep_$i.log 2>&1
  rc=$?; tail -2 gpurun_out/sweep_$i.log
  if [ $rc -ne 0 ]; then echo "run $i rc=$rc; stopping"; exit $rc; fi
done
