cd $GRAFT_REPO_ROOT
python -c "import torch; print(torch.cuda.get_device_name(0))"
timeout -k 10 1000 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 ${TESTK:+-k "$TESTK"} > gpurun_out/t1.log 2>&1
echo "pytest rc=$?"
tail -60 gpurun_out/t1.log
