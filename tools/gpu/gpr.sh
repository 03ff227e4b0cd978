#!/bin/bash
# (host-side helper, run from this container: never on the GPU box)
# run one gpurun call, retrying only while the pool reports no free slot / box (nothing ran, nothing charged)
OUT=$1; shift; TO=$1; shift
for i in $(seq 1 12); do
  timeout 2700 /usr/local/graft/bin/gpurun --timeout $TO -- "$@" > $OUT 2>&1
  if grep -q "backing off" $OUT || { grep -q "status=transient" $OUT && grep -q "nothing was charged\|no free box" $OUT; }; then
    sleep 150; continue
  fi
  break
done
