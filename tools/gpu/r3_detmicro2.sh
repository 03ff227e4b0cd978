#!/bin/bash
# bs1 detect conv shapes, graph-replayed: training forward (no epilogue) vs eval forward (BN + SiLU epilogue) vs vendor
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TUNE_GRAPH=1
timeout -k 10 300 python -u tools/gpu/tune_conv.py det fwd,infer,mm > gpurun_out/detmicro2.log 2>&1
