#!/bin/bash
# bf16 attention: two 32-query blocks per wave (w64, w64o) against the 8-wave bounded kernel: parity, A/B at
# config 2, effective clocks
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/w64clk
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc; return 0; }
run w64tests 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "attn or attention"
run w64ab 400 python tools/bench_kernels.py --only attention --variant bounded,w64,w64o --iters 8
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d gpurun_out/w64clk/attn -o k --output-format csv -- python tools/bench_kernels.py --only attention --iters 4 --variant bounded,w64,w64o > gpurun_out/w64clk/attn.log 2>&1
echo "pmc rc=$?"
exit 0
