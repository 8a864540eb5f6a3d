#!/bin/bash
# round-4 final tree, part A (B: gpu_r04_final2.sh): full GPU suite, smoke, the default bench line (CPU baseline
# included), the same bench under rocprofv3 --stats
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; grep "^{" "gpurun_out/$name.log" | cut -c1-250
  [ $rc -ne 0 ] && { tail -25 "gpurun_out/$name.log"; exit $rc; }; return 0; }
run r04f_gtests 600 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -rA
tail -1 gpurun_out/r04f_gtests.log
run r04f_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run r04f_bench 600 python bench.py
run r04f_prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r04f_prof -o k --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
exit 0
