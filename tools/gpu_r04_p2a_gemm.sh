#!/bin/bash
# p2a tests + GEMM variant 12 tests, kernel A/Bs (attention p2 / p2a / a16; GEMM 11 / 12 interleaved), config-2
# bench default and --qk-gamma 6
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 "gpurun_out/$name.log"
  [ $rc -ne 0 ] && { tail -40 "gpurun_out/$name.log"; exit $rc; }; return 0; }
run r04_p2a_tests 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_attention_fp8_gpu.py tests/test_pipeline_contract_gpu.py -k "attention or attn or contract or recorded or gemm" -x -q --timeout 120 --timeout-method thread
run r04_gemm12_ab 300 python tools/bench_kernels.py --only gemm --gemm-variants 11,12 --iters 10
run r04_p2a_ab 300 python tools/bench_kernels.py --only attention --variant p2,p2a,a16 --iters 10
run r04_bench_g6 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --qk-gamma 6
run r04_bench_def 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline
VP_GEMM_VARIANT=12 run r04_bench_g12 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline
exit 0
