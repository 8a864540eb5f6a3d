#!/bin/bash
# fp8 attention default = the skewed kernel (variant 5): fp8 tests, config-5 full-model parity, config-5 bench
# line, then variant 3 vs 5 interleaved at config 5's length
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_fp8_gpu.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/r04_skew_tests_final.log 2>&1 || { tail -30 gpurun_out/r04_skew_tests_final.log; exit 1; }
tail -1 gpurun_out/r04_skew_tests_final.log
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py -k "config5" -v -s --timeout 500 --timeout-method thread > gpurun_out/r04_skew_config5_model.log 2>&1 || { tail -30 gpurun_out/r04_skew_config5_model.log; exit 1; }
grep -E "config 5|passed|failed" gpurun_out/r04_skew_config5_model.log
timeout -k 10 600 python bench.py --config 5 --no-cpu-baseline > gpurun_out/r04_skew_bench_config5.log 2>&1 || { tail -30 gpurun_out/r04_skew_bench_config5.log; exit 1; }
grep "^{" gpurun_out/r04_skew_bench_config5.log | cut -c1-400
: > gpurun_out/r04_fp8_skew_ab.log
for i in 1 2; do
  timeout -k 10 200 python tools/bench_kernels.py --only attn8 --variant8 3,5 --video-tokens 46800 --iters 10 2>&1 | grep "attention fp8" >> gpurun_out/r04_fp8_skew_ab.log || exit 1
done
cat gpurun_out/r04_fp8_skew_ab.log
exit 0
