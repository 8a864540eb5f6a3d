#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (one counter block per run) on the GEMM and the bf16 attention at config-2 shapes:
# bash tools/pmc_traffic.sh [gemm variant] [kernels]
set -u
GV=${1:-13}
KS=${2:-"gemm attention"}
export TMPDIR=/tmp
mkdir -p gpurun_out
for K in $KS; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pmc_${K}_$C -o k --output-format csv -- python tools/bench_kernels.py --only $K --iters 2 --gemm-variants $GV --variant p2a > gpurun_out/pmc_${K}_$C.log 2>&1
    rc=$?; echo "pmc $K $C rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
