#!/bin/bash
# A/B of two builds of the library over a shape set: the in-tree build, then dmayolo/$ALTLIB swapped in
# (the box's copy of the tree is scratch).  SET / KINDS as in ab_conv.sh
cd $GRAFT_REPO_ROOT
L=dma-yolo_amd/dmayolo
for v in base alt; do
  [ $v = alt ] && cp $L/$ALTLIB $L/libdmayolo_hip.so
  echo "== $v"
  timeout -k 10 200 python tools/gpu/tune_conv.py ${SET:-dma} ${KINDS:-fwd,dgrad,wgrad} 2>&1 | grep -v amdgpu.ids || exit 1
done
