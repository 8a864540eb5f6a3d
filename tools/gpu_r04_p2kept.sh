#!/bin/bash
# p2 / p2a with kept LDS addresses: bit identity + interleaved A/B, then the attention GPU tests on the default
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/p2_kept_ab.py > gpurun_out/r04_p2kept_ab.log 2>&1 || { tail -20 gpurun_out/r04_p2kept_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_p2kept_ab.log
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention or attn" > gpurun_out/r04_p2kept_tests.log 2>&1 || { tail -30 gpurun_out/r04_p2kept_tests.log; exit 1; }
tail -1 gpurun_out/r04_p2kept_tests.log
exit 0
