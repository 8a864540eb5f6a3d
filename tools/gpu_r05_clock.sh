#!/bin/bash
# round 5: in-kernel clock + ablations of the bf16 attention (tools/attn_clock.py), the PMC of p2a, a short bench
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r05clk
L=videopainter_amd/_lib
step() {  # name timeout cmd...
  local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/r05clk/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"; tail -2 "gpurun_out/r05clk/$name.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step clk_a 240 env VP_HIP_LIB=$L/libvp_hip_clk.so python tools/attn_clock.py --label stock --variants p2a,p2,s16,a16
step nodma 120 env VP_HIP_LIB=$L/libvp_hip_clk_nodma.so python tools/attn_clock.py --label nodma --variants p2a
step noexp 120 env VP_HIP_LIB=$L/libvp_hip_clk_noexp.so python tools/attn_clock.py --label noexp --variants p2a
step noboth 120 env VP_HIP_LIB=$L/libvp_hip_clk_noboth.so python tools/attn_clock.py --label noboth --variants p2a
step clk_b 240 env VP_HIP_LIB=$L/libvp_hip_clk.so python tools/attn_clock.py --label stock2 --variants s16,a16,p2,p2a
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F32 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_LDS"
P3="SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_BRANCH"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  step pmc_p2a_p$i 180 rocprofv3 --pmc $P --kernel-trace -d gpurun_out/r05clk/pmc_p2a/p$i -o attn --output-format csv -- python tools/bench_kernels.py --only attention --iters 4 --variant p2a
done
step bench 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline
exit 0
