cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_bn_fuse.py -x -v -s -p no:cacheprovider --timeout 200 --timeout-method thread -k training > gpurun_out/t_bnf1.log 2>&1; echo rc=$?
