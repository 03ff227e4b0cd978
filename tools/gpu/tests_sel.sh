#!/bin/bash
# Selected GPU tests: TESTS="files..." TESTK="-k expr" (one pytest process, per-test timeout)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 ${TTIMEOUT:-500} python -u -m pytest ${TESTS:-tests} -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread ${TESTK:+-k "$TESTK"} > gpurun_out/tsel.log 2>&1
rc=$?; tail -30 gpurun_out/tsel.log; exit $rc
