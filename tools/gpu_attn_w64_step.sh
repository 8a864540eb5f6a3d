#!/bin/bash
# full GPU suite with the two-blocks-per-wave bounded attention as the default, then the config-2 step with it vs
# the 8-wave kernel (VP_ATTN_BOUNDED_MODE=w32), alternating runs, and a rocprof trace of the default
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc; tail -1 "gpurun_out/$name.log" | cut -c1-200; return 0; }
run gtests 600 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -rA
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_w64_1 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline
VP_ATTN_BOUNDED_MODE=w32 run bench_w32_1 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline
run bench_w64_2 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline
VP_ATTN_BOUNDED_MODE=w32 run bench_w32_2 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline
run prof_trace 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline
exit 0
