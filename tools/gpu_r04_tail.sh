#!/bin/bash
# GEMM tail split (the last partial round of tiles as split-K + reduce): tests, then calibration and config-2 benches
# alternating with VP_GEMM_NO_TAIL=1
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_training_gpu.py -k "gemm or transformer or branch or block or tail" -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_tail_tests.log 2>&1 || { tail -30 gpurun_out/r04_tail_tests.log; exit 1; }
tail -1 gpurun_out/r04_tail_tests.log
: > gpurun_out/r04_tail_ab.log
for i in 1 2; do
  echo "== no tail" >> gpurun_out/r04_tail_ab.log
  VP_GEMM_NO_TAIL=1 timeout -k 10 300 python tools/blas_calibration.py --rounds 1 --iters 10 2>&1 | grep -v amdgpu.ids >> gpurun_out/r04_tail_ab.log || exit 1
  echo "== tail" >> gpurun_out/r04_tail_ab.log
  timeout -k 10 300 python tools/blas_calibration.py --rounds 1 --iters 10 2>&1 | grep -v amdgpu.ids >> gpurun_out/r04_tail_ab.log || exit 1
done
grep -E "==|ff1 " gpurun_out/r04_tail_ab.log
: > gpurun_out/r04_tail_bench.log
for i in 1 2; do
  echo "== bench no tail" >> gpurun_out/r04_tail_bench.log
  VP_GEMM_NO_TAIL=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline 2>&1 | grep "^{" >> gpurun_out/r04_tail_bench.log || exit 1
  echo "== bench tail" >> gpurun_out/r04_tail_bench.log
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline 2>&1 | grep "^{" >> gpurun_out/r04_tail_bench.log || exit 1
done
python - <<'PY'
import json
lib = None
for line in open("gpurun_out/r04_tail_bench.log"):
    if line.startswith("=="): lib = line.strip(); continue
    d = json.loads(line)
    print(lib, round(d["value"], 4), "gemm ms", round(d["gemm_ms_per_step"], 1), "attn ms", round(d["attention_ms_per_step"], 1))
PY
exit 0
