#!/bin/bash
# round 3: fp8 attention LIN2 (pknorm packing) parity + interleaved A/B at config 5's length
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc; return 0; }
run r03_fp8_tests 400 python -u -m pytest tests/test_attention_fp8_gpu.py -x -v -s --timeout 300 --timeout-method thread
run r03_fp8_ab 400 python tools/bench_kernels.py --only attn8 --variant8 2,3,2,3 --video-tokens 46800 --iters 10
exit 0
