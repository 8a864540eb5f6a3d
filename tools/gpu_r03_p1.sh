#!/bin/bash
# one-wave-per-SIMD attention (p1): parity tests of the attention variants, then the interleaved A/B at config 2
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "attention" --timeout 120 \
  --timeout-method thread > gpurun_out/p1_tests.log 2>&1 || { tail -30 gpurun_out/p1_tests.log; exit 1; }
tail -3 gpurun_out/p1_tests.log
timeout -k 10 300 python -u tools/attn_ab.py --modes w64,p1 --rounds 5 --iters 20 > gpurun_out/p1_ab.log 2>&1
rc=$?; tail -4 gpurun_out/p1_ab.log; exit $rc
