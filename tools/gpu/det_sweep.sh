#!/bin/bash
# detect p50 (bs1, graph replay + NMS) under conv-library knob settings: CFGS="A=1,B=2 ..." CONFIG=dma-1536
cd $GRAFT_REPO_ROOT
for cfg in ${CFGS:-none}; do
  echo "== $cfg"
  env $(echo $cfg | tr ',' ' ') timeout -k 10 120 python tools/gpu/detect_only.py ${CONFIG:-dma-1536} 60 2>&1 | grep -v amdgpu.ids || exit 1
done
