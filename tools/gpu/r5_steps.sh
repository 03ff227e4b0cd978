#!/bin/bash
# Round 5: run named steps, each under its own limit, logs under gpurun_out/r5/<TAG>_<name>.log; a failing step ends
# the script.  STEPS="name:limit:command;;name:limit:command" (commands run by bash from the repo root), or STEPS_FILE=<file>.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r5
mkdir -p $OUT
TAG=${TAG:-s}
[ -n "$STEPS_FILE" ] && STEPS="$(cat $STEPS_FILE)"
( while sleep 50; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
IFS=$'\n'
for st in $(echo "$STEPS" | sed 's/;;/\n/g'); do
  name=${st%%:*}; rest=${st#*:}; lim=${rest%%:*}; cmd=${rest#*:}
  timeout -k 10 $lim bash -c "$cmd" > $OUT/${TAG}_$name.log 2>&1
  rc=$?; echo "$name rc=$rc"; tail -${TAILN:-6} $OUT/${TAG}_$name.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
