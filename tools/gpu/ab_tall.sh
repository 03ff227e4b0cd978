# tall 512x128 conv tile (DMY_CONV_TALL=1): parity of the conv tests on it, then per-shape A/B
cd $GRAFT_REPO_ROOT
DMY_CONV_TALL=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "fwd or dgrad" > gpurun_out/t_tall.log 2>&1
rc=$?; echo "tall conv tests rc=$rc"; tail -3 gpurun_out/t_tall.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for tv in 0 1; do
    echo "== set=c128 tall=$tv round=$r"
    DMY_CONV_TALL=$tv timeout -k 10 200 python tools/gpu/tune_conv.py c128 fwd,dgrad || exit 1
  done
done > gpurun_out/ab_tall.log 2>&1
echo "ab rc=$?"
