#!/bin/bash
# integer anchors: training-gradient accuracy (p2a vs p2), lse / attention kernel tests, LoRA + model tests, then the
# GEMM variant 13 A/B
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 "gpurun_out/$name.log"
  [ $rc -ne 0 ] && { grep -E "FAILED|Error" "gpurun_out/$name.log" | head -20; exit $rc; }; return 0; }
T=tests/test_training_gpu.py::test_branch_gradients_through_frozen_transformer
for v in p2a p2; do
  VP_ATTN_BOUNDED_MODE=$v timeout -k 10 200 python -u -m pytest $T -q -s --timeout 120 --timeout-method thread > gpurun_out/r04_train_int_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; grep -E "time_embedding.linear_1|output " gpurun_out/r04_train_int_$v.log
  [ $rc -gt 1 ] && exit $rc
done
run r04_attn_tests 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_backward_gpu.py -k "attn or attention or lse" -q --timeout 120 --timeout-method thread
run r04_lora_tests 600 python -u -m pytest tests/test_training_gpu.py tests/test_model_gpu.py tests/test_ulysses_gpu.py tests/test_pipeline_contract_gpu.py -v --timeout 120 --timeout-method thread
run r04_gemm13_tests 600 python -u -m pytest tests/test_kernels_gpu.py -k "gemm" -x -q --timeout 120 --timeout-method thread
run r04_gemm13_ab 300 python tools/bench_kernels.py --only gemm --gemm-variants 11,13 --iters 10
VP_GEMM_VARIANT=13 run r04_bench_g13 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline
run r04_bench_def2 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline
exit 0
