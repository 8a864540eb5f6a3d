set -u
# head_norm_rope with 4 heads per lane group (default) against one (libvp_hip_hnr1.so = the same sources with
# -DVP_HNR_HPG=1): interleaved processes, config-5 shape, speed + output digests; then the kernels' GPU tests.
mkdir -p gpurun_out/r06hnr
for i in 1 2 3; do
  timeout -k 10 120 python tools/bench_head_norm.py >> gpurun_out/r06hnr/ab.log 2>&1 || exit 2
  VP_HIP_LIB=videopainter_amd/_lib/libvp_hip_hnr1.so timeout -k 10 120 python tools/bench_head_norm.py >> gpurun_out/r06hnr/ab.log 2>&1 || exit 3
done
cat gpurun_out/r06hnr/ab.log
timeout -k 10 600 python -u -m pytest tests/test_attention_fp8_gpu.py tests/test_kernels_gpu.py tests/test_mx_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06hnr/tests.log 2>&1; rc=$?; tail -3 gpurun_out/r06hnr/tests.log; exit $rc
