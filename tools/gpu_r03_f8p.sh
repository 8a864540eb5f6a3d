#!/bin/bash
# round 3: the software-pipelined fp8 attention (VP_ATTN8_VARIANT=4): parity, then interleaved A/B against lin2 (3)
# at config 5's length
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"
  [ $rc -ne 0 ] && { tail -30 "gpurun_out/$name.log"; exit $rc; }; return 0; }
run r03_f8p_tests 300 python -u -m pytest tests/test_attention_fp8_gpu.py -x -v -s --timeout 120 --timeout-method thread -k "lin2"
grep -E "variant [34]|PASS|FAIL" gpurun_out/r03_f8p_tests.log | head -40
run r03_f8p_ab 300 python tools/bench_kernels.py --only attn8 --variant8 3,4,3,4 --video-tokens 46800 --iters 10
grep "attention fp8" gpurun_out/r03_f8p_ab.log
exit 0
