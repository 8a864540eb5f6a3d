#!/bin/bash
# training-step throughput on HEAD (branch trainable through the frozen transformer, config-2 shape)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python tools/bench_train.py --steps 3 --warmup 1 --classes > gpurun_out/r04_train_bench.log 2>&1; rc=$?
grep "^{" gpurun_out/r04_train_bench.log | cut -c1-600; exit $rc
