#!/bin/bash
# end-of-round measurements on the final tree (each step under its own limit; a failing step ends the script)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc; return 0; }
run gtests 600 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -rA
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py --steps 5 --warmup 2
run prof_trace 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline
run bench5 400 python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline
run bench4 500 python bench.py --config 4 --steps 2 --warmup 1
rm -rf gpurun_out/pmc_clock
bash tools/pmc_clock.sh > gpurun_out/pmc_clock.log 2>&1; echo "pmc_clock rc=$?"
exit 0
