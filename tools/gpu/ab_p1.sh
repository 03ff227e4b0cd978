#!/bin/bash
# 1x1 tile modes (DMY_P1_TILE 0..4) on the DMA-YOLO-l @1536 1x1 shapes, fwd + dgrad
cd $GRAFT_REPO_ROOT
AB_VAR=DMY_P1_TILE AB_VALS="0 1 3 4" SET=p1dma KINDS=fwd,dgrad bash tools/gpu/ab_conv.sh > gpurun_out/ab_p1.log 2>&1
rc=$?; cat gpurun_out/ab_p1.log; exit $rc
