#!/bin/bash
# p2 as the bounded default: kernel + model GPU tests, then the config-2 bench
set -u
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 "gpurun_out/$name.log"
  [ $rc -ne 0 ] && exit $rc; return 0; }
run p2_ktests 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread
run p2_bench 600 python bench.py
exit 0
