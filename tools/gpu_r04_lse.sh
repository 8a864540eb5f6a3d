#!/bin/bash
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "lse_matches" -v -s --timeout 120 --timeout-method thread > gpurun_out/r04_lse.log 2>&1
rc=$?; echo "lse rc=$rc"; grep -E "^lse|FAILED|passed|failed" gpurun_out/r04_lse.log | tail -30
exit 0
