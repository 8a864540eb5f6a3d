#!/bin/bash
# PMC passes (3) of the flash-attention backward at the training shape (tools/bench_attn_bwd.py):
#   bash tools/pmc_bwd.sh TAG      -> gpurun_out/pmc_bwd_TAG/p{1,2,3}
# then: python tools/pmc_report.py --dir gpurun_out/pmc_bwd_TAG --kernel bwd_dkdv_kernel (or bwd_dq_kernel)
set -u
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_LDS"
P3="SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_BRANCH"
TAG=${1:-base}
mkdir -p gpurun_out/pmc_bwd_$TAG
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $P --kernel-trace -d gpurun_out/pmc_bwd_$TAG/p$i -o ab --output-format csv -- python tools/bench_attn_bwd.py --iters 2 > gpurun_out/pmc_bwd_$TAG/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
