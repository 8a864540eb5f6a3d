#!/bin/bash
# wo_text branch (forward vs the reference golden, training gradients), fp8 GEMM default 13 tests, smoke
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300
  [ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" "gpurun_out/$name.log" | head -30; exit $rc; }; return 0; }
run r04_wotext_tests 600 python -u -m pytest tests/test_model_gpu.py tests/test_training_gpu.py tests/test_mx_gpu.py -k "wo_text or branch or mx" -v -s --timeout 120 --timeout-method thread
run r04_smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
exit 0
