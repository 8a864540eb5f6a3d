#!/bin/bash
# full GPU test suite, smoke, then a rocprof kernel trace of the config-5 bench (each step under its own limit)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc; return 0; }
run gtests 600 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -rA
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run prof5 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof5 -o bench5 --output-format csv -- python bench.py --config 5 --steps 2 --warmup 1 --no-cpu-baseline
exit 0
