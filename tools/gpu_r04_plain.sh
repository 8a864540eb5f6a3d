#!/bin/bash
# plain epilogues: unrolled row pass (libvp_hip.so) vs the per-row loop (libvp_hip_pslow.so): GEMM + model tests,
# then alternating calibration processes and config-2 benches
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L0=$PWD/videopainter_amd/_lib
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py tests/test_training_gpu.py -k "gemm or transformer" -x -q --timeout 300 --timeout-method thread > gpurun_out/r04_plain_tests.log 2>&1 || { tail -30 gpurun_out/r04_plain_tests.log; exit 1; }
tail -1 gpurun_out/r04_plain_tests.log
: > gpurun_out/r04_plain_ab.log
for i in 1 2; do
  for L in libvp_hip_pslow.so libvp_hip.so; do
    echo "== $L" >> gpurun_out/r04_plain_ab.log
    VP_HIP_LIB=$L0/$L timeout -k 10 300 python tools/blas_calibration.py --rounds 1 --iters 10 2>&1 | grep -v amdgpu.ids >> gpurun_out/r04_plain_ab.log || exit 1
  done
done
grep -E "==|qkv |ff1 " gpurun_out/r04_plain_ab.log
: > gpurun_out/r04_plain_bench.log
for L in libvp_hip_pslow.so libvp_hip.so libvp_hip_pslow.so libvp_hip.so; do
  echo "== bench $L" >> gpurun_out/r04_plain_bench.log
  VP_HIP_LIB=$L0/$L timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline 2>&1 | grep "^{" >> gpurun_out/r04_plain_bench.log || exit 1
done
python - <<'PY'
import json
lib = None
for line in open("gpurun_out/r04_plain_bench.log"):
    if line.startswith("=="): lib = line.split()[-1]; continue
    d = json.loads(line)
    print(lib, round(d["value"], 4), "gemm ms", round(d["gemm_ms_per_step"], 1), "attn ms", round(d["attention_ms_per_step"], 1))
PY
exit 0
