#!/bin/bash
# batch-1 detect A/B (graph-replayed eval forward + NMS, tools/gpu/detect_only.py): for each "name:ENV=V,..." in $AB
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
TAG=${TAG:-det}
( while sleep 50; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
for rep in 1 2; do
  for item in $AB; do
    name=${item%%:*}; envs=${item#*:}
    for cfg in ${CFGS:-dma-1536 v5s-640}; do
      out=$(env ${envs//,/ } timeout -k 10 200 python tools/gpu/detect_only.py $cfg ${ITERS:-200} 2>>gpurun_out/r4/detab_$TAG.err)
      rc=$?; echo "rep$rep $name ($envs) $cfg rc=$rc: $out" | tee -a gpurun_out/r4/detab_$TAG.log
      [ $rc -ne 0 ] && exit $rc
    done
  done
done
exit 0
