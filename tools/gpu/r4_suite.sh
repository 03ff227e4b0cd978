#!/bin/bash
# Round-4 full GPU suite (every failure listed, -rP keeps printed measurements) + smoke.  Own time limits per step.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r4
TAG=${TAG:-suite}
( while sleep 50; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
timeout -k 10 1050 python -u -m pytest ${TESTS:-tests} -m gpu -v -rP -p no:cacheprovider --timeout 600 --timeout-method thread \
    ${TESTK:+-k "$TESTK"} > gpurun_out/r4/tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/r4/tests_$TAG.log | tail -2; grep -E "^FAILED|^ERROR" gpurun_out/r4/tests_$TAG.log | head -30
[ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/smoke_$TAG.log 2>&1
src=$?; echo "smoke rc=$src"; tail -3 gpurun_out/r4/smoke_$TAG.log
exit $(( rc > src ? rc : src ))
