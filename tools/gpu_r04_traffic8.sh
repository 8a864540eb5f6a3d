#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the fp8 attention variant 3 (unskewed) at config 5's length, for comparison with the
# skewed default's 6.3x
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for C in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/r04_pmc_attn8v3_$C
  VP_ATTN8_VARIANT=3 timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/r04_pmc_attn8v3_$C -o k --output-format csv -- python tools/bench_kernels.py --only attn8 --iters 2 --video-tokens 46800 > gpurun_out/r04_pmc_attn8v3_$C.log 2>&1
  rc=$?; echo "attn8 v3 $C rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
