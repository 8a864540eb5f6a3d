#!/bin/bash
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attention or attn" > gpurun_out/ktests_attn.log 2>&1
rc=$?; echo "ktests rc=$rc"; tail -1 gpurun_out/ktests_attn.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/attn_mode_ab.py --rounds 3 > gpurun_out/attn_dot_ab.log 2>&1
rc=$?; echo "ab rc=$rc"; cat gpurun_out/attn_dot_ab.log | grep round; exit $rc
