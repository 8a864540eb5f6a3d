#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate) on the default bf16 attention (p2) at config 2
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for C in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/r03c_pmc_attention_$C
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/r03c_pmc_attention_$C -o k --output-format csv -- python tools/bench_kernels.py --only attention --iters 2 --variant bounded > gpurun_out/r03c_pmc_attention_$C.log 2>&1
  rc=$?; echo "$C rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
