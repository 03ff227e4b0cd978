#!/bin/bash
# Round-4 end-of-round GPU session: default bench (the driver's command), the 2-rank gloo rehearsal of --gpus 2 on this
# one GPU (the launch path of the 8-GPU run with the arena reducer), and the config-5 fp8 bench.  Each step has its
# own time limit; a failing step ends the script.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/r4
mkdir -p $OUT
TAG=${TAG:-final}
( while sleep 50; do echo "[hb] $(date +%T)"; done ) &
HB=$!
trap "kill $HB 2>/dev/null" EXIT
if [ -z "$NOBENCH" ]; then
  timeout -k 10 600 python bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARMUP:-5} > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
  rc=$?; echo "bench rc=$rc"; tail -c 600 $OUT/bench_$TAG.json; [ $rc -ne 0 ] && { tail -5 $OUT/bench_$TAG.err; exit $rc; }
fi
if [ -z "$NOGLOO" ]; then
  timeout -k 10 600 python bench.py --gpus 2 --backend gloo --steps 4 --warmup 2 --config dma-640 --also v5s-640 --no-detect \
      > $OUT/bench_gloo2_$TAG.json 2> $OUT/bench_gloo2_$TAG.err
  rc=$?; echo "gloo2 rc=$rc"; tail -c 400 $OUT/bench_gloo2_$TAG.json; [ $rc -ne 0 ] && { tail -5 $OUT/bench_gloo2_$TAG.err; exit $rc; }
fi
if [ -n "$C5" ]; then  # config 5 @1920 bs8, bf16 then the fp8 forward (delayed scaling)
  timeout -k 10 600 python bench.py --config c5-1920 --also none --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_c5_bf16_$TAG.json 2> $OUT/bench_c5_bf16_$TAG.err
  rc=$?; echo "c5 bf16 rc=$rc"; tail -c 400 $OUT/bench_c5_bf16_$TAG.json; [ $rc -ne 0 ] && exit $rc
  timeout -k 10 600 python bench.py --config c5-1920 --also none --fp8 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_c5_fp8_$TAG.json 2> $OUT/bench_c5_fp8_$TAG.err
  rc=$?; echo "c5 fp8 rc=$rc"; tail -c 400 $OUT/bench_c5_fp8_$TAG.json
fi
exit 0
