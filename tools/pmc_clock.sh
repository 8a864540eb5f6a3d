#!/bin/bash
# Effective clock per kernel (MI355X_MICROARCH.md 'DVFS give-back': GRBM_GUI_ACTIVE / 8 / dispatch wall time) for the
# config-2 GEMMs and bf16 attention and the config-5 fp8 attention; one rocprofv3 --pmc run per kernel set.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/pmc_clock
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d $OUT/gemm -o k --output-format csv -- python tools/bench_kernels.py --only gemm --iters 4 --gemm-variants 11 > $OUT/gemm.log 2>&1
rc=$?; echo "gemm rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d $OUT/attn -o k --output-format csv -- python tools/bench_kernels.py --only attention --iters 4 --variant bounded > $OUT/attn.log 2>&1
rc=$?; echo "attn rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d $OUT/attn8 -o k --output-format csv -- python tools/bench_kernels.py --only attn8 --iters 4 --video-tokens 46800 > $OUT/attn8.log 2>&1
rc=$?; echo "attn8 rc=$rc"; exit $rc
