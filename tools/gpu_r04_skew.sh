#!/bin/bash
# skewed fp8 attention (VP_ATTN8_VARIANT 5 / 6): fp8 tests (bit identity with variant 3 first), then interleaved
# kernel timings at config 5's length
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_fp8_gpu.py -x -v -s --timeout 120 --timeout-method thread -k "skewed" > gpurun_out/r04_skew_tests.log 2>&1 || { tail -30 gpurun_out/r04_skew_tests.log; exit 1; }
tail -1 gpurun_out/r04_skew_tests.log
timeout -k 10 400 python -u -m pytest tests/test_attention_fp8_gpu.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/r04_skew_tests_all.log 2>&1 || { tail -30 gpurun_out/r04_skew_tests_all.log; exit 1; }
tail -1 gpurun_out/r04_skew_tests_all.log
: > gpurun_out/r04_skew_ab.log
for i in 1 2; do
  timeout -k 10 200 python tools/bench_kernels.py --only attn8 --variant8 3,5,6 --video-tokens 46800 --iters 10 2>&1 | grep "attention fp8" >> gpurun_out/r04_skew_ab.log || exit 1
done
cat gpurun_out/r04_skew_ab.log
exit 0
