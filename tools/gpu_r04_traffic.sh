#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate runs) on the shipped attention kernels: bf16 p2a at config 2, fp8 (skewed,
# variant 5) at config 5's length
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for C in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/r04_pmc_attn_$C gpurun_out/r04_pmc_attn8_$C
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/r04_pmc_attn_$C -o k --output-format csv -- python tools/bench_kernels.py --only attention --iters 2 --variant p2a > gpurun_out/r04_pmc_attn_$C.log 2>&1
  rc=$?; echo "attn $C rc=$rc"; [ $rc -ne 0 ] && exit $rc
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/r04_pmc_attn8_$C -o k --output-format csv -- python tools/bench_kernels.py --only attn8 --iters 2 --video-tokens 46800 > gpurun_out/r04_pmc_attn8_$C.log 2>&1
  rc=$?; echo "attn8 $C rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
