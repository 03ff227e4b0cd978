#!/bin/bash
# Round 5 parity diagnostics: per-layer product vs bf16_sink emulation (dx rounded as stored) at the bench shapes,
# with the fp16 autocast emulation per layer (config 5's C3TR); oracle trajectory determinism + fp64 pin; the
# DMA-YOLO-l distribution test; memory / optimizer tests.  Each step has its own limit; a failure ends the script.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r5
mkdir -p $OUT
TAG=${TAG:-par}
( while sleep 50; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
step() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > $OUT/${TAG}_$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; tail -4 $OUT/${TAG}_$name.log
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step mem 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_gpu_memory.py tests/test_gpu_optim.py
step lay_c5 600 env DIAG_FP16=1 python -u tools/gpu/diag_modules.py yolov5l-xs-tr-cbam-spp-bifpn.yaml 1920 2 all
step lay_dma 600 python -u tools/gpu/diag_modules.py yolov5l-ca-sppfcspc-bifpn-scconv.yaml 1536 2 all
step trajdet 600 python -u tools/gpu/diag_traj_det.py 6
step dist 900 python -u -m pytest -x -v -s --timeout 850 --timeout-method thread -m gpu tests/test_gpu_bench_shape.py -k "bf16_vs_oracle and scconv"
exit 0
