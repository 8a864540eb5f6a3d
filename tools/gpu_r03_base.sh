#!/bin/bash
# round-3 opening check on a fresh box: smoke + config-2 bench (each step under its own limit)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc; return 0; }
run r03_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run r03_bench_base 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline
exit 0
