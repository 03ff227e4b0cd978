#!/bin/bash
# Round 6: how much of the first bench-shape parity test is MIOpen building kernels for the fp32 oracle
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r6
mkdir -p $OUT
export MIOPEN_USER_DB_PATH=/tmp/miopen_a MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_a
timeout -k 10 300 python tools/gpu/miopen_probe.py yolov5l-xs-tr-cbam-spp-bifpn.yaml 1920 2 >> $OUT/miopen_probe.log 2>&1 || exit $?
export MIOPEN_USER_DB_PATH=/tmp/miopen_b MIOPEN_CUSTOM_CACHE_DIR=/tmp/miopen_b MIOPEN_FIND_MODE=FAST
timeout -k 10 300 python tools/gpu/miopen_probe.py yolov5l-xs-tr-cbam-spp-bifpn.yaml 1920 2 >> $OUT/miopen_probe.log 2>&1 || exit $?
cat $OUT/miopen_probe.log
