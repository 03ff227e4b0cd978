cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_optim.py tests/test_gpu_model.py tests/test_gpu_determinism.py tests/test_gpu_ddp.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/t_arena.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t_arena.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/t_arena.log | head; exit $rc; }
timeout -k 10 300 python bench.py --config v5s-640 --also none --steps 20 --warmup 5 --no-cpu-baseline --no-detect > gpurun_out/b_v5s.log 2>&1; rc=$?; echo "bench rc=$rc"; head -c 400 gpurun_out/b_v5s.log
timeout -k 10 200 python tools/gpu/diag_copies.py > gpurun_out/diag.log 2>&1; echo "diag rc=$?"; head -25 gpurun_out/diag.log
