# rocprofv3 kernel stats of the config-5 bench with fp8 forward convs (short run)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fp8 -o run -- python bench.py --config c5-1920 --also none --steps 3 --warmup 1 --no-cpu-baseline --no-detect --fp8 > gpurun_out/prof_fp8.log 2>&1
rc=$?; echo "rc=$rc"; f=$(find gpurun_out/prof_fp8 -name "*kernel_stats.csv" | head -1); echo $f; head -40 "$f" | cut -d, -f1-4 | cut -c1-150
