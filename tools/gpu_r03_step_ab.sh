#!/bin/bash
# round 3: in-step A/B of the bf16 attention forms (alternating config-2 bench runs on one box)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
  for m in w64 s16 a16; do
    VP_ATTN_BOUNDED_MODE=$m timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r03_stepab_${m}_$i.log 2>&1
    rc=$?; echo "$m $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
