#!/bin/bash
# fp8 GEMM parity, then config-2 bench + rocprof stats and config-5 bench (each step under its own limit)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc; return 0; }
run mxtests 300 python -u -m pytest tests/test_mx_gpu.py tests/test_attention_fp8_gpu.py -x -q --timeout 120 --timeout-method thread
run bench 400 python bench.py --steps 5 --warmup 2 --no-cpu-baseline
run prof_trace 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline
run bench5 400 python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline
exit 0
