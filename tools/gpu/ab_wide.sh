# wide 256x256 conv tile (DMY_CONV_WIDE=<min cols>): parity of the conv tests on it, then per-shape A/B
cd $GRAFT_REPO_ROOT
DMY_CONV_WIDE=128 timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "fwd or dgrad" > gpurun_out/t_wide.log 2>&1
rc=$?; echo "wide conv tests rc=$rc"; tail -3 gpurun_out/t_wide.log; [ $rc -ne 0 ] && exit $rc
for set in dma s2 v5s; do
  for r in 1 2; do
    for wv in 0 128; do
      echo "== set=$set wide=$wv round=$r"
      DMY_CONV_WIDE=$wv timeout -k 10 200 python tools/gpu/tune_conv.py $set fwd,dgrad || exit 1
    done
  done
done > gpurun_out/ab_wide.log 2>&1
echo "ab rc=$?"
