#!/bin/bash
# round 3: w64 back as the bounded default (+ its k2_full instance): attention tests, resample model tests,
# config-4 with w64+hint vs s16+hint, config-2 default
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc; return 0; }
run r03_c4tests 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread -k "attn or attention or partition or resample"
run r03_c4_w64 500 python bench.py --config 4 --steps 2 --warmup 1
VP_ATTN_BOUNDED_MODE=s16 run r03_c4_s16 500 python bench.py --config 4 --steps 2 --warmup 1
run r03_c2_w64 400 python bench.py --steps 6 --warmup 2 --no-cpu-baseline
exit 0
