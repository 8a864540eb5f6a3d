#!/bin/bash
# One full config-2 step of the oracle on the GPU box's host cores (bf16), with a per-minute progress stamp under
# gpurun_out/ (the step prints nothing for ~7 min)
set -u
mkdir -p gpurun_out
( while true; do date >> gpurun_out/cpu_full_step.tick; sleep 50; done ) &
TICK=$!
timeout -k 10 1000 python bench.py --cpu-baseline-only --cpu-full-step > gpurun_out/cpu_full_step.json 2> gpurun_out/cpu_full_step.err
rc=$?
kill $TICK
echo "cpu full step rc=$rc"; cat gpurun_out/cpu_full_step.json
exit $rc
