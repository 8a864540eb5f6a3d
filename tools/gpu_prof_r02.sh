#!/bin/bash
# rocprofv3 kernel traces of the config-2 step with the unstaggered (5) and staggered (11) GEMM main loops
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
for V in 11 5; do
  VP_GEMM_VARIANT=$V timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_v$V -o bench --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_v$V.log 2>&1
  rc=$?; echo "prof v$V rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
