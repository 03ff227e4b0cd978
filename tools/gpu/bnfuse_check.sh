# fused producer-BN reduce in the data-grad epilogue: its tests, the model / determinism / DDP suites, then the bench
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_bn_fuse.py tests/test_gpu_conv.py tests/test_gpu_model.py tests/test_gpu_bench_shape.py tests/test_gpu_determinism.py tests/test_gpu_ddp.py tests/test_gpu_optim.py -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/t_bnf.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "fused|worst" gpurun_out/t_bnf.log | head -5; tail -3 gpurun_out/t_bnf.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/t_bnf.log | head -20; exit $rc; }
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-detect > gpurun_out/b_bnf.log 2>&1; rc=$?; echo "bench rc=$rc"; python -c "
import json; d=json.loads(open('gpurun_out/b_bnf.log').read().strip().splitlines()[-1]); print('dma', d['value'], d['ms_per_step'], 'v5s', d['at_640']['value'], d['at_640']['ms_per_step'])"
exit $rc
