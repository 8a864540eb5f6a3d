#!/bin/bash
# VAE conv V2 (VP_CONV_PIPE=2, default) vs the round-3 pipe (1): VAE GPU tests on V2, then the 5b VAE bench
# alternating the two in separate processes
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_vae_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/r04_conv_tests.log 2>&1 || { tail -30 gpurun_out/r04_conv_tests.log; exit 1; }
tail -1 gpurun_out/r04_conv_tests.log
: > gpurun_out/r04_conv_ab.log
for P in 1 2 1 2; do
  VP_CONV_PIPE=$P timeout -k 10 300 python tools/bench_vae.py 2>&1 | grep "^{" | sed "s/^/pipe$P /" >> gpurun_out/r04_conv_ab.log || exit 1
done
cut -c1-700 gpurun_out/r04_conv_ab.log
exit 0
