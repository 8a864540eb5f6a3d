#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/p1_debug.py > gpurun_out/p1_debug.log 2>&1 || { tail -20 gpurun_out/p1_debug.log; exit 1; }
grep "^p1" gpurun_out/p1_debug.log
timeout -k 10 300 python -u tools/attn_ab.py --modes w64,p1 --rounds 4 --iters 20 > gpurun_out/p1_ab.log 2>&1
rc=$?; tail -3 gpurun_out/p1_ab.log; exit $rc
