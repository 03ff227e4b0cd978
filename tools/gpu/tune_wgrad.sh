#!/bin/bash
# wgrad split-K target sweep (one process per target; the library reads DMY_WGRAD_TARGET once)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for t in ${TARGETS:-512 1024 2048}; do
  echo "== DMY_WGRAD_TARGET=$t"
  DMY_WGRAD_TARGET=$t timeout -k 10 300 python tools/gpu/tune_conv.py ${SET:-dma} wgrad || exit $?
done
