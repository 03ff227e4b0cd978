#!/bin/bash
# bs1 detect p50 over the split-K plan knobs (target blocks in % of the CUs, fewest K steps per split)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for v in "DMY_SPLITK_PCT=200" "DMY_SPLITK_PCT=100" "DMY_SPLITK_PCT=150" "DMY_SPLITK_PCT=300" "DMY_SPLITK_PCT=400" \
         "DMY_SPLITK_MINK=4" "DMY_SPLITK_MINK=8" "DMY_SPLITK_MAXM=1"; do
  for cfg in dma-1536 v5s-640; do
    env $v timeout -k 10 120 python -u tools/gpu/detect_only.py $cfg 60 2>/dev/null | sed "s/^/$v /" \
      | tee -a gpurun_out/splitab.log || exit 1
  done
done
