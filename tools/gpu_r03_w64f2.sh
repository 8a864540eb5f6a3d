#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/p1_debug.py > gpurun_out/w64f_debug.log 2>&1 || { tail -20 gpurun_out/w64f_debug.log; exit 1; }
grep "^w64f" gpurun_out/w64f_debug.log
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "attention" --timeout 120 \
  --timeout-method thread > gpurun_out/w64f_tests.log 2>&1 || { tail -30 gpurun_out/w64f_tests.log; exit 1; }
tail -2 gpurun_out/w64f_tests.log
timeout -k 10 300 python -u tools/attn_ab.py --modes w64,w64f --rounds 8 --iters 20 > gpurun_out/w64f_ab.log 2>&1
rc=$?; tail -3 gpurun_out/w64f_ab.log; exit $rc
