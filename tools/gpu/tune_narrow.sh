#!/bin/bash
# narrow wgrad: v2 (DMY_WGRAD_NARROW=0) vs LDS-DMA narrow tiles at several split-K block targets
cd $GRAFT_REPO_ROOT
echo "== v2"; DMY_WGRAD_NARROW=0 timeout -k 10 120 python tools/gpu/tune_conv.py narrow wgrad 2>&1 | grep -v amdgpu || exit 1
echo "== narrow model"; timeout -k 10 120 python tools/gpu/tune_conv.py narrow wgrad 2>&1 | grep -v amdgpu || exit 1
for t in ${TARGETS:-256 512 1024 2048 4096}; do
  echo "== narrow target $t"; DMY_WGRAD_TARGET=$t timeout -k 10 120 python tools/gpu/tune_conv.py narrow wgrad 2>&1 | grep -v amdgpu || exit 1
done
