#!/bin/bash
# p2 with the two row-sum MFMAs spread (libvp_hip_rs.so) against the default library, alternating processes
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/rs_ab.log
for i in 1 2 3; do
  for L in libvp_hip.so libvp_hip_rs.so libvp_hip_pr.so; do
    echo "== $L" >> gpurun_out/rs_ab.log
    VP_HIP_LIB=$PWD/videopainter_amd/_lib/$L timeout -k 10 120 python -u tools/attn_ab.py --modes p2 --rounds 3 --iters 20 2>&1 | grep "median" >> gpurun_out/rs_ab.log || exit 1
  done
done
cat gpurun_out/rs_ab.log
timeout -k 10 500 python bench.py --config 4 --steps 2 --warmup 1 > gpurun_out/r03b_bench_c4.log 2>&1; echo "c4 rc=$?"
tail -1 gpurun_out/r03b_bench_c4.log | cut -c1-400
