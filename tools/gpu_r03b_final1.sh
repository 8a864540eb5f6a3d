#!/bin/bash
# round 3 (second session) end-of-round measurements, part 1: full GPU suite, smoke, default bench (with the CPU baseline), the
# rocprofv3 kernel trace of the same bench command
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc; return 0; }
run r03b_gtests 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -rA
run r03b_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run r03b_bench 600 python bench.py
rm -rf gpurun_out/r03b_prof
run r03b_prof_trace 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r03b_prof -o bench --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline
exit 0
