#!/bin/bash
# round 3: full GPU suite (LDS-flag fix, 4-wave GEMM variant 20 in the GEMM parity tests), GEMM A/B 11 vs 20,
# config-2 benches (default, GEMM v20, gamma-6 qk-norm), config-4 bench
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc; return 0; }
run r03_gtests2 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -rA
run r03_gemm_ab 300 python tools/bench_kernels.py --only gemm --gemm-variants 11,20 --iters 10
run r03_bench_c2 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline
VP_GEMM_VARIANT=20 run r03_bench_c2_g20 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline
run r03_bench_c2_g6 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --qk-gamma 6
run r03_bench_c4 500 python bench.py --config 4 --steps 2 --warmup 1
exit 0
