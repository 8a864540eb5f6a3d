#!/bin/bash
# PMC passes for bounded attention variants (VP_ATTN_BOUNDED_MODE names): bash tools/pmc_attn_p1.sh w64 p1
set -u
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_LDS"
P3="SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_BRANCH"
for V in "$@"; do
  mkdir -p gpurun_out/pmc_b_$V
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace -d gpurun_out/pmc_b_$V/p$i -o attn --output-format csv -- python tools/bench_kernels.py --only attention --iters 2 --variant $V > gpurun_out/pmc_b_$V/p$i.log 2>&1
    rc=$?; echo "$V pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
