#!/bin/bash
# round 3: the resample processor's null keys in closed form (k2_len + l_extra): kernel + model tests, config 4 with
# and without it, config 2 default
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc; return 0; }
run r03_null_tests 500 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -v --timeout 300 --timeout-method thread -k "null or k2_len or k2_full or resample or anchored or large_gamma or tail_split"
run r03_null_ab 300 python tools/null_ab.py --rounds 3
run r03_c4_null 500 python bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline
VP_RESAMPLE_NULLMASS=0 run r03_c4_keys 500 python bench.py --config 4 --steps 2 --warmup 1 --no-cpu-baseline
run r03_c2 400 python bench.py --steps 6 --warmup 2 --no-cpu-baseline
exit 0
