#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/p1_debug.py > gpurun_out/w64f_debug.log 2>&1 || { tail -20 gpurun_out/w64f_debug.log; exit 1; }
grep "^w64f" gpurun_out/w64f_debug.log
timeout -k 10 300 python -u tools/attn_ab.py --modes w64,w64f --rounds 6 --iters 20 > gpurun_out/w64f_ab.log 2>&1
rc=$?; tail -3 gpurun_out/w64f_ab.log; exit $rc
