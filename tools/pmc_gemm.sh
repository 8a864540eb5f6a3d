#!/bin/bash
# PMC passes on the GEMM kernel (one main-loop variant per invocation): bash tools/pmc_gemm.sh <variant>
set -u
export TMPDIR=/tmp
V=$1
mkdir -p gpurun_out/pmc_gemm_v$V
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INST_LEVEL_VMEM"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace -d gpurun_out/pmc_gemm_v$V/p$i -o gemm --output-format csv -- python tools/bench_kernels.py --only gemm --iters 2 --gemm-variants $V > gpurun_out/pmc_gemm_v$V/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
