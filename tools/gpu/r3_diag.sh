#!/bin/bash
# bf16 parity attribution (tools/gpu/diag_precision.py) on yolov5s @640 bs16 and DMA-YOLO-l @1536 bs2
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u tools/gpu/diag_precision.py yolov5s.yaml 640 16 > gpurun_out/diag_prec_v5s.log 2>&1
rc=$?; echo "v5s rc=$rc"; tail -3 gpurun_out/diag_prec_v5s.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 750 python -u tools/gpu/diag_precision.py yolov5l-ca-sppfcspc-bifpn-scconv.yaml 1536 2 > gpurun_out/diag_prec_dma.log 2>&1
rc=$?; echo "dma rc=$rc"; tail -3 gpurun_out/diag_prec_dma.log; exit $rc
