#!/bin/bash
# MFMA T5 attention: T5 tests, then the encoder bench with the MFMA (default) and the scalar kernel, and a kernel
# stats profile of the default
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_t5_gpu.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/r04_t5_tests.log 2>&1 || { tail -30 gpurun_out/r04_t5_tests.log; exit 1; }
grep -E "rel|passed|failed" gpurun_out/r04_t5_tests.log | tail -14
for A in scalar mfma scalar mfma; do
  VP_T5_ATTN=$A timeout -k 10 200 python tools/bench_t5.py --iters 10 2>&1 | grep "^{" | sed "s/^/$A /" >> gpurun_out/r04_t5_bench.log || exit 1
done
cut -c1-330 gpurun_out/r04_t5_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_t5_prof -o t5 --output-format csv -- python tools/bench_t5.py --iters 5 > gpurun_out/r04_t5_prof.log 2>&1 || exit 1
exit 0
