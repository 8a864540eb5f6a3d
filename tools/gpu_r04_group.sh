#!/bin/bash
# GEMM tile-group size A/B (VP_GEMM_GROUP: M-tiles per group of the grouped tile order): tests, then alternating
# calibration processes
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_mx_gpu.py -k "gemm or mx" -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_group_tests.log 2>&1 || { tail -30 gpurun_out/r04_group_tests.log; exit 1; }
tail -1 gpurun_out/r04_group_tests.log
VP_GEMM_GROUP=8 timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "gemm_layout_exact or gemm_bias_random or tail or gated_inject" -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_group8_tests.log 2>&1 || { tail -30 gpurun_out/r04_group8_tests.log; exit 1; }
tail -1 gpurun_out/r04_group8_tests.log
: > gpurun_out/r04_group_ab.log
for i in 1 2; do
  for G in 4 8 2 6; do
    echo "== group $G" >> gpurun_out/r04_group_ab.log
    VP_GEMM_GROUP=$G timeout -k 10 300 python tools/blas_calibration.py --rounds 1 --iters 10 2>&1 | grep -v amdgpu.ids >> gpurun_out/r04_group_ab.log || exit 1
  done
done
cat gpurun_out/r04_group_ab.log
exit 0
