#!/bin/bash
# Round 6: run a subset of GPU tests (TESTS, default: the round-6 parity / DDP / detect changes) with per-test
# durations and printed output into gpurun_out/r6/<TAG>.log
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r6
TAG=${TAG:-tests}
TESTS=${TESTS:-"tests/test_gpu_model.py::test_graphed_detect_after_call_recapture tests/test_gpu_ddp.py tests/test_gpu_mha.py tests/test_gpu_bench_shape.py"}
timeout -k 10 ${TLIM:-1080} python -u -m pytest $TESTS -x -v -s -m gpu --timeout ${PTO:-600} --timeout-method thread \
  --durations=40 > gpurun_out/r6/$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -60 gpurun_out/r6/$TAG.log
exit $rc
