#!/bin/bash
# QKV epilogue (qk-norm + RoPE with operands loaded ahead, permlane reductions): kernel/model parity, GEMM
# calibration with the step epilogues, config-2 bench (each step under its own limit)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc; return 0; }
run ktests 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_attention_fp8_gpu.py -x -q --timeout 200 --timeout-method thread
run mtests 600 python -u -m pytest tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread
run blascal 400 python tools/blas_calibration.py --rounds 2 --iters 10
run bench 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline
exit 0
