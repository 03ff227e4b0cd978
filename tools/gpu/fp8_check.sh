# fp8 forward conv: parity tests, then config 5 bench bf16 vs fp8 (short runs, no CPU baseline / detect)
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_fp8.py -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/t_fp8.log 2>&1
rc=$?; echo "fp8 tests rc=$rc"; grep -E "PASS|FAIL|Error|level rel|loss bf16|assert" gpurun_out/t_fp8.log | head -40; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config c5-1920 --also none --steps 5 --warmup 2 --no-cpu-baseline --no-detect --layer-report > gpurun_out/b_c5_bf16.log 2> gpurun_out/b_c5_bf16.err; rc=$?; echo "bf16 rc=$rc"; head -c 300 gpurun_out/b_c5_bf16.log; echo; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --config c5-1920 --also none --steps 5 --warmup 2 --no-cpu-baseline --no-detect --layer-report --fp8 > gpurun_out/b_c5_fp8.log 2> gpurun_out/b_c5_fp8.err; rc=$?; echo "fp8 rc=$rc"; head -c 300 gpurun_out/b_c5_fp8.log; echo
exit $rc
