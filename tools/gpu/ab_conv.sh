#!/bin/bash
# A/B of a conv-library knob over a shape set: AB_VAR=<env var> AB_VALS="0 1" SET=dma KINDS=fwd,dgrad,wgrad
cd $GRAFT_REPO_ROOT
for v in ${AB_VALS:-0 1}; do
  echo "== ${AB_VAR:-DMY_CONV_BUF}=$v"
  env ${AB_VAR:-DMY_CONV_BUF}=$v timeout -k 10 200 python tools/gpu/tune_conv.py ${SET:-dma} ${KINDS:-fwd,dgrad,wgrad} 2>&1 | grep -v amdgpu.ids || exit 1
done
