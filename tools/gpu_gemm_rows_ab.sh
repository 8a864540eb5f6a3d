#!/bin/bash
# GEMM epilogue row-pass batching: kernel parity, then the block's GEMMs with their real epilogues, new vs abl/old
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ktests.log 2>&1
rc=$?; echo "ktests rc=$rc"; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  timeout -k 10 200 python tools/gemm_block_shapes.py > gpurun_out/gbs_new_$r.log 2>&1; rc=$?; echo "new $r rc=$rc"; [ $rc -ne 0 ] && exit $rc
  (cd abl/old && timeout -k 10 200 python tools/gemm_block_shapes.py > ../../gpurun_out/gbs_old_$r.log 2>&1); rc=$?; echo "old $r rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
