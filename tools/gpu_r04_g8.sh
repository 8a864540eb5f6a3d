#!/bin/bash
# MX-FP8 GEMMs at config 5's shapes: grouped tile order A/B (VP_GEMM_GROUP 4 = default, 2, 8, 16), separate processes,
# interleaved
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r04_g8_ab.log
for r in 1 2; do
  for G in 4 2 8 16; do
    VP_GEMM_GROUP=$G timeout -k 10 200 python tools/bench_kernels.py --only mx --video-tokens 46800 --iters 10 2>&1 | grep "gemm mxfp8" | sed "s/^/group=$G /" >> gpurun_out/r04_g8_ab.log || exit 1
  done
done
cat gpurun_out/r04_g8_ab.log
exit 0
