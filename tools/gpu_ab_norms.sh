# A/B of the AdaLN kernel variants (VP_ADALN_VARIANT 0 / 1), alternating processes, + the bit-exactness tests
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_mx_gpu.py -x -q --timeout 120 --timeout-method thread -k "adaln or modulate" > gpurun_out/ab/adaln_tests.log 2>&1; echo tests rc=$?

for r in 1 2; do
  for v in 0; do
    VP_ADALN_VARIANT=$v timeout -k 10 120 python tools/bench_kernels.py --only norms --iters 20 > gpurun_out/ab/norms_v${v}_$r.log 2>&1 || exit 1
  done
done
grep -H "adaln" gpurun_out/ab/norms_v*.log | grep -v json; tail -1 gpurun_out/ab/adaln_tests*.log
