#!/bin/bash
# bs1 detect conv shapes, graph-replayed GPU time per launch: default plan, FILL tiles, conv_sk, vendor GEMM (1x1)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TUNE_GRAPH=1
for v in "" "DMY_V3_FILL=1" "DMY_SK=1"; do
  echo "== ${v:-default}" | tee -a gpurun_out/detmicro.log
  env $v timeout -k 10 200 python -u tools/gpu/tune_conv.py det infer >> gpurun_out/detmicro.log 2>&1 || exit 1
done
echo "== vendor" >> gpurun_out/detmicro.log
timeout -k 10 200 python -u tools/gpu/tune_conv.py det mm >> gpurun_out/detmicro.log 2>&1
