#!/bin/bash
# GEMM variant 13 as the default: tests (bf16 + fp8 main loops), config-5 fp8 GEMM A/B (5 vs 13), the config-2 bench
# under rocprofv3 stats, then GEMM PMC (busy / waits / clock) and traffic passes on variant 13
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-400
  [ $rc -ne 0 ] && { grep -E "FAILED|Error" "gpurun_out/$name.log" | head -20; exit $rc; }; return 0; }
run r04_g13_tests 600 python -u -m pytest tests/test_mx_gpu.py tests/test_kernels_gpu.py -k "gemm or mx" -q --timeout 120 --timeout-method thread
run r04_c5_g8v5 500 python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline
VP_GEMM8_VARIANT=13 run r04_c5_g8v13 500 python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline
run r04_bench_g13_prof 500 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_g13_prof -o k --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
run r04_pmc_gemm13 400 bash tools/pmc_gemm.sh 13
run r04_traffic_gemm13 400 bash tools/pmc_traffic.sh 13 gemm
exit 0
