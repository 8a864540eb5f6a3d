#!/bin/bash
# fp8 attention: linear-code P (variant 2) against exp2 + RNE (variant 1): parity, kernel A/B at config-5 shape,
# model-level fp8 tests, config-5 bench, then the PMC passes of the default kernel (each step under its own limit)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc; return 0; }
run f8tests 400 python -u -m pytest tests/test_attention_fp8_gpu.py -x -v -s --timeout 200 --timeout-method thread
run f8ab 300 python tools/bench_kernels.py --only attn8 --variant8 1,2 --iters 6 --video-tokens 46800
run f8model 600 python -u -m pytest tests/test_model_gpu.py -x -v -s -k "fp8 or config1 or config5" --timeout 300 --timeout-method thread
run bench5 400 python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline
bash tools/pmc_attn8.sh > gpurun_out/pmc_attn8.log 2>&1; echo "pmc rc=$?"
exit 0
