#!/bin/bash
# round 3 (third session) final tree: full GPU suite, smoke, config-2 bench, rocprof trace, config-5 bench
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc; return 0; }
run r03d_gtests 900 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -rA
run r03d_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run r03d_bench 600 python bench.py
exit 0
