#!/bin/bash
# unfused-LoRA GPU tests (training backward, sub-ulp update, processors, contract), then the GEMM variant 13 A/B
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 "gpurun_out/$name.log"
  [ $rc -ne 0 ] && { tail -60 "gpurun_out/$name.log"; exit $rc; }; return 0; }
run r04_lora_tests 600 python -u -m pytest tests/test_training_gpu.py tests/test_model_gpu.py tests/test_ulysses_gpu.py tests/test_pipeline_contract_gpu.py -x -v --timeout 120 --timeout-method thread
run r04_gemm13_tests 600 python -u -m pytest tests/test_kernels_gpu.py -k "gemm" -x -q --timeout 120 --timeout-method thread
run r04_gemm13_ab 300 python tools/bench_kernels.py --only gemm --gemm-variants 11,13 --iters 10
VP_GEMM_VARIANT=13 run r04_bench_g13 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline
run r04_bench_def2 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline
exit 0
