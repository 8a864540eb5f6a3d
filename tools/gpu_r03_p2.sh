#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/p1_debug.py > gpurun_out/p2_debug.log 2>&1 || { tail -20 gpurun_out/p2_debug.log; exit 1; }
grep -E "^p[12]" gpurun_out/p2_debug.log
timeout -k 10 300 python -u tools/attn_ab.py --modes w64f,p2,p1 --rounds 6 --iters 20 > gpurun_out/p2_ab.log 2>&1
rc=$?; tail -3 gpurun_out/p2_ab.log; exit $rc
