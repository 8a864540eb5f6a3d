#!/bin/bash
set -u
mkdir -p gpurun_out
for r in 1 2; do
  for L in hip ab_prio; do
    VP_HIP_LIB=videopainter_amd/_lib/libvp_$L.so timeout -k 10 200 python tools/bench_kernels.py --only attention --variant bounded --iters 20 > gpurun_out/attnab_${L}_$r.log 2>&1
    rc=$?; echo "$L $r rc=$rc"; [ $rc -ne 0 ] && exit $rc
    grep "attention bounded" gpurun_out/attnab_${L}_$r.log
  done
done
exit 0
