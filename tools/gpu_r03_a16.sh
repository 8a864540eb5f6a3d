#!/bin/bash
# round 3: anchored-softmax attention (a16) next to s16 / w64 / lazy: parity incl. large-gamma and late-jump paths,
# interleaved A/B at config 2
set -u
export TMPDIR=/tmp
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"
  [ $rc -ne 0 ] && exit $rc; return 0; }
run a16tests 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 200 --timeout-method thread -k "attn or attention" -s
run a16ab 400 python tools/bench_kernels.py --only attention --variant w64,s16,a16,lazy,s16,a16 --iters 10
exit 0
