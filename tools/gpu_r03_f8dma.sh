#!/bin/bash
# default fp8 attention (lin2) with 32-bit LDS DMA addresses (libvp_hip.so) vs the generic-pointer form
# (libvp_hip_f8old.so): fp8 tests on the new library, then alternating processes at config 5's length
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_attention_fp8_gpu.py -x -v -s --timeout 120 --timeout-method thread > gpurun_out/r03_f8dma_tests.log 2>&1 || { tail -30 gpurun_out/r03_f8dma_tests.log; exit 1; }
tail -1 gpurun_out/r03_f8dma_tests.log
: > gpurun_out/r03_f8dma_ab.log
for i in 1 2 3; do
  for L in libvp_hip_f8old.so libvp_hip.so; do
    echo "== $L" >> gpurun_out/r03_f8dma_ab.log
    VP_HIP_LIB=$PWD/videopainter_amd/_lib/$L timeout -k 10 120 python tools/bench_kernels.py --only attn8 --variant8 3 --video-tokens 46800 --iters 10 2>&1 | grep "attention fp8" >> gpurun_out/r03_f8dma_ab.log || exit 1
  done
done
cat gpurun_out/r03_f8dma_ab.log
