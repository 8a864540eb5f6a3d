#!/bin/bash
# PMC passes on the fp8 attention variants (VP_ATTN8_VARIANT values) at config 5's length:
# bash tools/pmc_attn8_ab.sh 3 4; summary: python tools/pmc_b_summary.py f8v3 f8v4
set -u
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_LDS"
P3="SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_BRANCH"
for V in "$@"; do
  mkdir -p gpurun_out/pmc_b_f8v$V
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    VP_ATTN8_VARIANT=$V timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace -d gpurun_out/pmc_b_f8v$V/p$i -o attn --output-format csv -- python tools/bench_kernels.py --only attn8 --iters 2 --video-tokens 46800 > gpurun_out/pmc_b_f8v$V/p$i.log 2>&1
    rc=$?; echo "$V pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
python tools/pmc_b_summary.py $(for V in "$@"; do echo -n "f8v$V "; done) > gpurun_out/pmc_attn8_ab_summary.txt
cat gpurun_out/pmc_attn8_ab_summary.txt
exit 0
