#!/bin/bash
# round 3: bf16 attention variants (parity incl. the partitioned resample segment), interleaved A/B + clocks
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/ab1clk
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc; return 0; }
run ab1tests 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "attn or attention or partition"
run ab1model 400 python -u -m pytest tests/test_model_gpu.py -x -v --timeout 300 --timeout-method thread -k "resample" -s
run ab1 500 python tools/attn_ab.py --modes w64,s16,s16i,a16,a16i --unbounded lazy --rounds 5 --iters 20
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace -d gpurun_out/ab1clk/attn -o k --output-format csv -- python tools/attn_ab.py --modes w64,s16,s16i,a16,a16i --rounds 1 --iters 3 > gpurun_out/ab1clk/attn.log 2>&1
echo "pmc rc=$?"
exit 0
