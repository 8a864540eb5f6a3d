#!/bin/bash
# fp8 attention: the row-sum selector tuple from a resident pair (4 v_mov_b64): fp8 tests, config-5 parity, 3 vs 5 timings
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_fp8_gpu.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/r04_sel4_tests.log 2>&1 || { tail -30 gpurun_out/r04_sel4_tests.log; exit 1; }
tail -1 gpurun_out/r04_sel4_tests.log
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py -k "config5" -v -s --timeout 500 --timeout-method thread > gpurun_out/r04_sel4_config5_model.log 2>&1 || { tail -30 gpurun_out/r04_sel4_config5_model.log; exit 1; }
grep -E "config 5|passed|failed" gpurun_out/r04_sel4_config5_model.log
: > gpurun_out/r04_sel4_ab.log
for i in 1 2; do
  timeout -k 10 200 python tools/bench_kernels.py --only attn8 --variant8 3,5 --video-tokens 46800 --iters 10 2>&1 | grep "attention fp8" >> gpurun_out/r04_sel4_ab.log || exit 1
done
cat gpurun_out/r04_sel4_ab.log
exit 0
