#!/bin/bash
# PMC passes on the fp8 attention kernel (attn_fwd_fp8) at config-5 shapes (B=2, 48 heads, 226 + 46800 tokens):
# three SQ instruction-mix passes + FETCH_SIZE / WRITE_SIZE, each its own rocprofv3 run (one counter set per run).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/pmc_attn8
mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_LDS"
P3="SQ_INSTS_SALU SQ_INST_LEVEL_VMEM"
i=0
for P in "$P1" "$P2" "$P3" FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace -d $OUT/p$i -o attn8 --output-format csv -- python tools/bench_kernels.py --only attn8 --iters 2 --video-tokens 46800 > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($P) rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
