#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "linear_small" -v --timeout 120 --timeout-method thread > gpurun_out/r04_ls_tests.log 2>&1 || { tail -30 gpurun_out/r04_ls_tests.log; exit 1; }
tail -1 gpurun_out/r04_ls_tests.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_ls_prof -o k --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r04_ls_prof.log 2>&1 || { tail -20 gpurun_out/r04_ls_prof.log; exit 1; }
grep "^{" gpurun_out/r04_ls_prof.log | cut -c1-200
grep -E "linear_small" gpurun_out/r04_ls_prof/k_kernel_stats.csv | cut -c1-200
exit 0
