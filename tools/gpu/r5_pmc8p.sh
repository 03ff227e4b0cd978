#!/bin/bash
# Round 5: PMC of the 3x3 wide tiles, 2-stage loop (DMY_W8P=0) vs the half-tile pipeline (DMY_W8P=2), forward only,
# shape set 'one' (3x3 256 @96^2 and 1024 @48^2, bs32): MFMA busy, LDS bank conflicts, wait / issue breakdown.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5
for m in 0 2; do
  for pass in mfma stall; do
    DMY_W8P=$m PMCTAG=r5_w8p${m} PMCPASSES=$pass PMCTIMEOUT=120 \
      PMCCMD="python $GRAFT_REPO_ROOT/tools/gpu/tune_conv.py one fwd" bash tools/gpu/pmc.sh || exit $?
  done
done
for m in 0 2; do python tools/pmc_summary.py gpurun_out/pmc_r5_w8p$m >> gpurun_out/r5/pmc_w8p.txt 2>&1; done
head -40 gpurun_out/r5/pmc_w8p.txt
exit 0
