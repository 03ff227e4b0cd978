# A/B of the small-grid LDS-DMA tiles (DMY_V3_FILL) on the bs1 detect path: p50 latency + kernel traces
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT/dma-yolo_amd TMPDIR=/tmp
for r in 1 2; do for v in 0 1; do for c in dma-1536 v5s-640; do
  echo -n "FILL=$v run$r "; DMY_V3_FILL=$v timeout -k 10 120 python tools/gpu/detect_only.py $c 60 2>/dev/null | grep p50 || exit 1
done; done; done
for v in 0 1; do
  (cd /tmp && DMY_V3_FILL=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/fill$v -o run \
     --output-format csv -- python $GRAFT_REPO_ROOT/tools/gpu/detect_only.py dma-1536 30 > /dev/null 2>&1) || exit 1
done
echo done
