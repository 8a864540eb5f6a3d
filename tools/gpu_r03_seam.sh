#!/bin/bash
# p2 with the seam-step MFMA order (libvp_hip_seam.so) against the default library, alternating processes
set -o pipefail
mkdir -p gpurun_out
VP_HIP_LIB=$PWD/videopainter_amd/_lib/libvp_hip_seam.so VP_ATTN_BOUNDED_MODE=p2 timeout -k 10 120 python -u tools/p1_debug.py > gpurun_out/seam_debug.log 2>&1 || { tail -5 gpurun_out/seam_debug.log; exit 1; }
grep "^p2" gpurun_out/seam_debug.log
: > gpurun_out/seam_ab.log
for i in 1 2 3; do
  for L in libvp_hip.so libvp_hip_seam.so; do
    echo "== $L" >> gpurun_out/seam_ab.log
    VP_HIP_LIB=$PWD/videopainter_amd/_lib/$L timeout -k 10 120 python -u tools/attn_ab.py --modes p2 --rounds 3 --iters 20 2>&1 | grep "median" >> gpurun_out/seam_ab.log || exit 1
  done
done
cat gpurun_out/seam_ab.log | grep -v "^{"
