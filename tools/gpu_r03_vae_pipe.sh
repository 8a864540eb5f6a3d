#!/bin/bash
# VAE conv: counted-vmcnt pipeline (default) vs the 2-stage ring (VP_CONV_PIPE=0), VAE GPU tests; then the p1
# attention A/B.  Every GPU step under its own limit.
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_vae_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/vae_tests.log 2>&1
rc=$?; echo "vae tests rc=$rc"; tail -2 gpurun_out/vae_tests.log; [ $rc -ne 0 ] && exit $rc
for P in 1 0 1 0; do
  VP_CONV_PIPE=$P timeout -k 10 200 python tools/bench_vae.py --iters 2 > gpurun_out/vae_bench_p$P.log 2>&1
  rc=$?; echo "vae bench pipe=$P rc=$rc"; [ $rc -ne 0 ] && exit $rc
  tail -1 gpurun_out/vae_bench_p$P.log
done
bash tools/gpu_r03_p1b.sh
