#!/bin/bash
# T5 encoder: the split-K partial-bytes cap (VP_GEMM_SPLIT_PART 1 = default, 2 lets the o projection fill the chip),
# interleaved encoder timings, T5 tests under 2, a kernel trace under 2
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r04_t5split_ab.log
for P in 1 2 1 2 1 2; do
  VP_GEMM_SPLIT_PART=$P timeout -k 10 200 python tools/bench_t5.py --iters 10 2>&1 | grep "^{" | sed "s/^/part=$P /" >> gpurun_out/r04_t5split_ab.log || exit 1
done
cut -c1-300 gpurun_out/r04_t5split_ab.log
VP_GEMM_SPLIT_PART=2 timeout -k 10 300 python -u -m pytest tests/test_t5_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_t5split_tests.log 2>&1 || { tail -30 gpurun_out/r04_t5split_tests.log; exit 1; }
tail -1 gpurun_out/r04_t5split_tests.log
VP_GEMM_SPLIT_PART=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_t5split_prof -o t5 --output-format csv -- python tools/bench_t5.py --iters 5 > gpurun_out/r04_t5split_prof.log 2>&1 || exit 1
exit 0
