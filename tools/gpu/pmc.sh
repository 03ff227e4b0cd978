#!/bin/bash
# PMC passes (one counter group per run, each under its own kill-timeout) over a command given as
# PMCCMD (default: the DMA-YOLO-l @1536 conv shape set).  Output: gpurun_out/pmc_<tag>_<pass>/
#   pass mfma : MFMA-busy / LDS counters (SQ block) + GRBM_GUI_ACTIVE (clock)
#   pass stall: where waves wait (parked on s_waitcnt / barrier vs issue stalls vs active) + MFMA-busy
#   pass fetch: FETCH_SIZE        pass write: WRITE_SIZE   (cannot share a pass: TCC slots)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${PMCTAG:-conv}
CMD=${PMCCMD:-"python $GRAFT_REPO_ROOT/tools/gpu/tune_conv.py dma"}
declare -A GROUPS_=(
  [mfma]="SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
  [stall]="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
  [fetch]="FETCH_SIZE"
  [write]="WRITE_SIZE"
)
for pass in ${PMCPASSES:-mfma fetch write}; do
  out=$GRAFT_REPO_ROOT/gpurun_out/pmc_${TAG}_${pass}
  (cd /tmp && timeout -s KILL ${PMCTIMEOUT:-150} rocprofv3 --kernel-trace --pmc ${GROUPS_[$pass]} -d $out -o run \
      --output-format csv -- $CMD > $out.log 2>&1)
  rc=$?
  echo "pmc pass $pass rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out.log; exit $rc; fi
done
