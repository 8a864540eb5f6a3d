#!/bin/bash
# round 3: the 16x16x32 bf16 attention (s16) against the 32x32x16 two-blocks-per-wave default (w64): parity,
# interleaved A/B at config 2, effective clocks
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/s16clk
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc; return 0; }
run s16tests 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "attn or attention"
run s16ab 400 python tools/bench_kernels.py --only attention --variant w64,s16,w64,s16 --iters 8
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d gpurun_out/s16clk/attn -o k --output-format csv -- python tools/bench_kernels.py --only attention --iters 4 --variant w64,s16 > gpurun_out/s16clk/attn.log 2>&1
echo "pmc rc=$?"
exit 0
