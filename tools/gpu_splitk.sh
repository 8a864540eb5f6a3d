#!/bin/bash
set -u
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc; tail -1 "gpurun_out/$name.log" | cut -c1-400; return 0; }
run ktests 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_t5_gpu.py -x -q --timeout 120 --timeout-method thread
run t5bench 300 python tools/bench_t5.py --iters 5
exit 0
