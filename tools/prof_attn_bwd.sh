#!/bin/bash
# rocprofv3 kernel stats of the attention backward at the training shape (tools/bench_attn_bwd.py)
set -e
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof_attn_bwd}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o ab --output-format csv -- python3 tools/bench_attn_bwd.py --iters 3 > $OUT.log 2>&1
