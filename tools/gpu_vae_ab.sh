#!/bin/bash
# VAE conv A/B (tap-hoisted gather vs per-K-tile decode) + VAE GPU tests; every GPU step under its own limit
set -u
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_vae_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/vae_tests.log 2>&1
rc=$?; echo "vae tests rc=$rc"; [ $rc -ne 0 ] && exit $rc
for H in 1 0 1; do
  VP_CONV_HOIST=$H timeout -k 10 200 python tools/bench_vae.py --iters 2 > gpurun_out/vae_bench_h$H.log 2>&1
  rc=$?; echo "vae bench hoist=$H rc=$rc"; [ $rc -ne 0 ] && exit $rc
  tail -1 gpurun_out/vae_bench_h$H.log
done
exit 0
