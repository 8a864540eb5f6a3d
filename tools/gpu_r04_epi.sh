#!/bin/bash
# GEMM epilogue A/B: libvp_hip.so (vector bias loads + RoPE quads prefetched a fragment ahead) against the round-3
# form (libvp_hip_epiold.so, -DVP_GEMM_EPI_OLD=1) and the gated epilogue with its residual rows loaded before the LDS
# image (libvp_hip_rpre.so, -DVP_GEMM_EPI_RPRE=1): GEMM tests on each, alternating calibration processes, benches
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
L0=$PWD/videopainter_amd/_lib
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "gemm or linear_small" -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_epi_tests.log 2>&1 || { tail -30 gpurun_out/r04_epi_tests.log; exit 1; }
tail -1 gpurun_out/r04_epi_tests.log
VP_HIP_LIB=$L0/libvp_hip_rpre.so timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "gemm" -x -q --timeout 120 --timeout-method thread > gpurun_out/r04_rpre_tests.log 2>&1 || { tail -30 gpurun_out/r04_rpre_tests.log; exit 1; }
tail -1 gpurun_out/r04_rpre_tests.log
: > gpurun_out/r04_epi_ab.log
for i in 1 2; do
  for L in libvp_hip_epiold.so libvp_hip.so libvp_hip_rpre.so; do
    echo "== $L" >> gpurun_out/r04_epi_ab.log
    VP_HIP_LIB=$L0/$L timeout -k 10 300 python tools/blas_calibration.py --rounds 1 --iters 10 2>&1 | grep -v amdgpu.ids >> gpurun_out/r04_epi_ab.log || exit 1
  done
done
cat gpurun_out/r04_epi_ab.log
: > gpurun_out/r04_epi_bench.log
for L in libvp_hip_epiold.so libvp_hip.so libvp_hip_rpre.so libvp_hip_epiold.so libvp_hip.so libvp_hip_rpre.so; do
  echo "== bench $L" >> gpurun_out/r04_epi_bench.log
  VP_HIP_LIB=$L0/$L timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline 2>&1 | grep "^{" >> gpurun_out/r04_epi_bench.log || exit 1
done
python - <<'PY'
import json
lib = None
for line in open("gpurun_out/r04_epi_bench.log"):
    if line.startswith("=="): lib = line.split()[-1]; continue
    d = json.loads(line)
    print(lib, round(d["value"], 4), "gemm ms", round(d["gemm_ms_per_step"], 1), "attn ms", round(d["attention_ms_per_step"], 1))
PY
exit 0
