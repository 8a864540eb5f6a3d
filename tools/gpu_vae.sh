#!/bin/bash
# VAE measurement on one MI355X: bench (untiled, tiled) + rocprofv3 kernel stats of the untiled decode/encode.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_vae.py --iters 2 > gpurun_out/vae_bench.log 2>&1; rc=$?; echo "vae bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_vae.py --iters 1 --tiled > gpurun_out/vae_bench_tiled.log 2>&1; rc=$?; echo "vae tiled rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_vae -o vae --output-format csv -- python tools/bench_vae.py --iters 1 > gpurun_out/prof_vae.log 2>&1; rc=$?; echo "vae prof rc=$rc"
exit $rc
