#!/bin/bash
# One GPU session: tests, smoke, bench. Every GPU step has its own time limit; a crash/timeout stops the script.
set -u
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for step in "$@"; do
  case $step in
    ktests) run ktests 600 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -rA ;;
    mtests) run mtests 900 python -u -m pytest tests/test_model_gpu.py -v --timeout 300 --timeout-method thread -rA ;;
    gtests) run gtests 1150 python -u -m pytest tests -v -m gpu --timeout 300 --timeout-method thread -rA ;;
    ftests) run ftests 600 python -u -m pytest tests/test_attention_fp8_gpu.py tests/test_mx_gpu.py -v --timeout 300 --timeout-method thread -rA ;;
    smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench)  run bench 900 python bench.py --steps 5 --warmup 2 ;;
    benchq) run bench 900 python bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
    kbench) run kbench 300 python tools/bench_kernels.py --iters 5 ;;
    prof)   export TMPDIR=/tmp; run prof_trace 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    blasprof) export TMPDIR=/tmp; run blasprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/blasprof -o blas --output-format csv -- python tools/blas_calibration.py --rounds 1 --iters 3 ;;
    pmc)    export TMPDIR=/tmp; run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o attn --output-format csv -- python tools/bench_kernels.py --only attention --iters 2 && run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o attn --output-format csv -- python tools/bench_kernels.py --only attention --iters 2 ;;
  esac
done
