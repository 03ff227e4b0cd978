#!/bin/bash
# bench A/B on one box: for each "name:ENV=V,ENV2=V2" in $AB, `python bench.py $ARGS` under that environment
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
TAG=${TAG:-bab}
ARGS=${ARGS:-"--config dma-1536 --also none --steps 10 --warmup 3 --no-cpu-baseline --no-detect"}
( while sleep 50; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
for item in $AB; do
  name=${item%%:*}; envs=${item#*:}
  env ${envs//,/ } timeout -k 10 400 python bench.py $ARGS > gpurun_out/r4/benchab_${TAG}_$name.json 2> gpurun_out/r4/benchab_${TAG}_$name.err
  rc=$?
  echo "$name ($envs) rc=$rc $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" gpurun_out/r4/benchab_${TAG}_$name.json 2>/dev/null)"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/r4/benchab_${TAG}_$name.err; exit $rc; }
done
exit 0
