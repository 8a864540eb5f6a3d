#!/bin/bash
# round-4 measurement: the default bench line (with the CPU baseline), then the same command under rocprofv3 stats
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; grep "^{" "gpurun_out/$name.log" | cut -c1-300
  [ $rc -ne 0 ] && { tail -20 "gpurun_out/$name.log"; exit $rc; }; return 0; }
run r04m_bench 900 python bench.py
run r04m_prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r04m_prof -o k --output-format csv -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline
exit 0
