#!/bin/bash
# tap-fused weight-grad: correctness (conv + determinism tests), A/B timing vs the column-tile kernels, DMA layer report
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_determinism.py -k "wgrad or det or run_twice" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t_wgrad.log 2>&1
rc=$?; echo "wgrad tests rc=$rc"; tail -3 gpurun_out/t_wgrad.log
[ $rc -ne 0 ] && exit $rc
for set in dma v5s narrow; do
  AB_VAR=DMY_WGRAD_TAP SET=$set KINDS=wgrad bash tools/gpu/ab_conv.sh > gpurun_out/ab_tap_$set.log 2>&1 || exit 1
  cat gpurun_out/ab_tap_$set.log
done
[ -n "$NOREPORT" ] && exit 0
timeout -k 10 400 python bench.py --config dma-1536 --also none --steps 3 --warmup 1 --layer-report --no-cpu-baseline --no-detect > gpurun_out/dma_layers.log 2> gpurun_out/dma_layers.err
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/dma_layers.log
exit $rc
