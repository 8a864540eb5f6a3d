#!/bin/bash
# config-5 bench line on HEAD (fp8 attention without scratch), then the same under rocprofv3 --stats
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; grep "^{" "gpurun_out/$name.log" | cut -c1-250
  [ $rc -ne 0 ] && { tail -25 "gpurun_out/$name.log"; exit $rc; }; return 0; }
run r04g_c5line 300 python bench.py --config 5 --no-cpu-baseline
run r04g_c5 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r04g_c5prof -o k --output-format csv -- python bench.py --config 5 --no-cpu-baseline
exit 0
