#!/bin/bash
# Round-6 HEAD measurement refresh: GEMMs interleaved beside hipBLASLt, the QKV GEMM's FETCH / WRITE traffic and its
# SQ passes, the attention backward's SQ passes, the fp8 attention's SQ + traffic passes (each pass its own run).
set -u
mkdir -p gpurun_out/r06pmc
timeout -k 10 300 python tools/blas_calibration.py --rounds 3 --iters 10 > gpurun_out/r06pmc/blas.log 2>&1 || exit 1
tail -4 gpurun_out/r06pmc/blas.log
bash tools/pmc_traffic.sh 13 gemm || exit 2
bash tools/pmc_gemm.sh 13 || exit 3
bash tools/pmc_bwd.sh r06 || exit 4
bash tools/pmc_attn8.sh || exit 5
mv gpurun_out/pmc_gemm_FETCH_SIZE gpurun_out/pmc_gemm_WRITE_SIZE gpurun_out/pmc_gemm_v13 gpurun_out/pmc_bwd_r06 gpurun_out/pmc_attn8 gpurun_out/r06pmc/
