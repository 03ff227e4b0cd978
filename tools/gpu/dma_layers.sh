cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py --config dma-1536 --also none --steps 3 --warmup 1 --layer-report --no-cpu-baseline --no-detect > gpurun_out/dma_layers.log 2> gpurun_out/dma_layers.err
rc=$?; echo "bench rc=$rc"; tail -c 1500 gpurun_out/dma_layers.log; tail -3 gpurun_out/dma_layers.err
exit $rc
