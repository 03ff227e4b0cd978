#!/bin/bash
# A/B of one test under library knobs: for each "name:ENV=V ENV2=V2" in $AB run $T with that environment.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
TAG=${TAG:-ab}
( while sleep 50; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
for item in $AB; do
  name=${item%%:*}; envs=${item#*:}
  env ${envs//,/ } timeout -k 10 ${TT:-400} python -u -m pytest $T -v -s -p no:cacheprovider --timeout 380 \
      --timeout-method thread > gpurun_out/r4/ab_${TAG}_$name.log 2>&1
  rc=$?; echo "$name ($envs) rc=$rc"; grep -E "grad-norm vector|worst layers|largest grad-norm|passed|failed" gpurun_out/r4/ab_${TAG}_$name.log | head -8
  [ $rc -ge 2 ] && exit $rc
done
exit 0
