#!/bin/bash
# fp8 attention: parity tests (default kernel, then the VALU-sum variant), interleaved A/B, config-5 bench
set -u
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc; return 0; }
run f8tests 300 python -u -m pytest tests/test_attention_fp8_gpu.py -x -q --timeout 120 --timeout-method thread
VP_ATTN8_VARIANT=1 run f8tests_v1 300 python -u -m pytest tests/test_attention_fp8_gpu.py -x -q --timeout 120 --timeout-method thread
run attn8_ab 300 python tools/bench_kernels.py --only attn8 --iters 10 --variant8 1,2
grep -h "attention_fp8\|attn8\|fp8" gpurun_out/attn8_ab.log | tail -6
run bench5 600 python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline
tail -1 gpurun_out/bench5.log | cut -c1-400
exit 0
