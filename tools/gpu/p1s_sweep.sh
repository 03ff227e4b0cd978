#!/bin/bash
# launch-shape sweep of the 1x1 streaming GEMM (DMY_P1S_NTH / _LDS / _BPC) against the LDS-DMA tiles
cd $GRAFT_REPO_ROOT
for cfg in "DMY_P1S=0" "DMY_P1S_NTH=256 DMY_P1S_LDS=64 DMY_P1S_BPC=3" "DMY_P1S_NTH=256 DMY_P1S_LDS=40 DMY_P1S_BPC=4" \
           "DMY_P1S_NTH=512 DMY_P1S_LDS=80 DMY_P1S_BPC=2" "DMY_P1S_NTH=512 DMY_P1S_LDS=160 DMY_P1S_BPC=1" \
           "DMY_P1S_NTH=1024 DMY_P1S_LDS=160 DMY_P1S_BPC=1" "DMY_P1S_NTH=256 DMY_P1S_LDS=64 DMY_P1S_BPC=8"; do
  echo "== $(echo $cfg | tr ' ' ',')"
  env $cfg timeout -k 10 200 python tools/gpu/tune_conv.py ${SET:-p1s} fwd,dgrad 2>&1 | grep -v amdgpu.ids || exit 1
done
