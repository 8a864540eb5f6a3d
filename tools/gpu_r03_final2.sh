#!/bin/bash
# round 3 end-of-round measurements, part 2: FETCH_SIZE / WRITE_SIZE passes (attention, GEMM), config 4 and 5 benches
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc; return 0; }
for K in attention gemm; do
  for C in FETCH_SIZE WRITE_SIZE; do
    rm -rf gpurun_out/r03_pmc_${K}_$C
    run r03_pmc_${K}_$C 300 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/r03_pmc_${K}_$C -o k --output-format csv -- python tools/bench_kernels.py --only $K --iters 2 --gemm-variants 11 --variant bounded
  done
done
run r03_bench_c4 500 python bench.py --config 4 --steps 2 --warmup 1
run r03_bench_c5 500 python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline
exit 0
