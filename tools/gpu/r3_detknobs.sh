#!/bin/bash
# bs1 detect p50 under the small-M routing knobs, re-measured after the eval-epilogue fix
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in "DMY_NONE=0" "DMY_P1P_SMALL=1" "DMY_SK=1" "DMY_V3_FILL=1" "DMY_SPLITK_P1=1" "DMY_P1P_EP=1"; do
  for cfg in dma-1536 v5s-640; do
    env $v timeout -k 10 120 python -u tools/gpu/detect_only.py $cfg 60 2>/dev/null | sed "s/^/$v /" \
      | tee -a gpurun_out/detknobs.log || exit 1
  done
done
