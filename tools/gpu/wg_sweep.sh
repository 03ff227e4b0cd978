#!/bin/bash
# weight-grad knob sweep over a shape set: CFGS="A=1,B=2 ..." SET=v5s
cd $GRAFT_REPO_ROOT
for cfg in ${CFGS:-X=0}; do
  echo "== $cfg"
  env $(echo $cfg | tr ',' ' ') timeout -k 10 200 python tools/gpu/tune_conv.py ${SET:-v5s} wgrad 2>&1 | grep -v amdgpu.ids || exit 1
done
