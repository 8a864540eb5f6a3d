#!/bin/bash
# GEMM epilogue rework: kernel + model parity, then K-scan of the new library against the previous commit's (abl/old)
set -u
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc; return 0; }
run ktests 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread
run mtests 600 python -u -m pytest tests/test_model_gpu.py tests/test_training_gpu.py tests/test_t5_gpu.py -x -q --timeout 300 --timeout-method thread
for r in 1 2; do
  run kscan_new_$r 200 python tools/gemm_kscan.py --iters 10
  (cd abl/old && timeout -k 10 200 python tools/gemm_kscan.py --iters 10 > ../../gpurun_out/kscan_old_$r.log 2>&1); rc=$?; echo "old $r rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
