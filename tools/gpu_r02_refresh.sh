#!/bin/bash
# measurements of the §8f rows and the other configs on the current tree (each step under its own limit)
set -u
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc; tail -1 "gpurun_out/$name.log" | cut -c1-600; return 0; }
run t5bench 300 python tools/bench_t5.py --iters 5
run blascal 400 python tools/blas_calibration.py --rounds 2 --iters 10
run trainbench 400 python tools/bench_train.py --steps 3 --warmup 1
run bench4 500 python bench.py --config 4 --steps 2 --warmup 1
exit 0
