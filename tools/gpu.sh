#!/bin/bash
# The one GPU-session launcher (the only one: the per-experiment launchers of rounds 1-4 are folded into it):
#
#   gpurun -- bash tools/gpu.sh TAG 'name[@timeout]=command' ['name[@timeout]=command' ...]
#
# Each step runs under its own `timeout -k 10` (default 300 s), writes gpurun_out/TAG/<name>.log, and prints its exit
# code and last line.  The session stops at the first failing step (a fault, abort, time-limit kill or test failure
# ends it: nothing more runs on the GPU after it).  Shortcuts for the usual steps:
#   gtests   the whole -m gpu suite          smoke   __graft_entry__.smoke()
#   bench    bench.py --steps 5 --warmup 2   prof    bench.py under rocprofv3 --kernel-trace --stats
set -u
export TMPDIR=/tmp
TAG=$1
shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for spec in "$@"; do
  if [[ "$spec" == *=* ]]; then head=${spec%%=*}; cmd=${spec#*=}; else head=$spec; cmd=""; fi
  name=${head%%@*}
  to=300
  [ "$head" != "$name" ] && to=${head#*@}
  if [ -z "$cmd" ]; then
    case "$name" in
      gtests) cmd="python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -rA" ;;
      smoke) cmd="python -c 'import __graft_entry__ as g; g.smoke()'" ;;
      bench) cmd="python bench.py --steps 5 --warmup 2" ;;
      prof) cmd="rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline" ;;
      *) echo "unknown step $name"; exit 2 ;;
    esac
  fi
  t0=$(date +%s)
  timeout -k 10 "$to" bash -c "$cmd" > "$OUT/$name.log" 2>&1
  rc=$?
  echo "$name rc=$rc ($(( $(date +%s) - t0 )) s): $(tail -1 "$OUT/$name.log" | cut -c1-300)"
  if [ $rc -ne 0 ]; then
    echo "stopping after $name (rc=$rc)"
    exit $rc
  fi
done
exit 0
