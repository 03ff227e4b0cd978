# eltwise kernels: module / model parity suites, then the bench
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_modules.py tests/test_gpu_model.py tests/test_gpu_tal.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/t_elt.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/t_elt.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/t_elt.log | head; exit $rc; }
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-detect > gpurun_out/b_elt.log 2>&1; rc=$?; echo "bench rc=$rc"; python -c "
import json; d=json.loads(open('gpurun_out/b_elt.log').read().strip().splitlines()[-1]); print('dma', d['value'], d['ms_per_step'], 'v5s', d['at_640']['value'], d['at_640']['ms_per_step'])"
