set -e
mkdir -p gpurun_out/ab
for r in 1 2; do
  timeout -k 10 120 python tools/bench_kernels.py --only attention --iters 10 > gpurun_out/ab/attn_def_$r.log 2>&1
  VP_HIP_LIB=abl/noslp/libvp_hip.so timeout -k 10 120 python tools/bench_kernels.py --only attention --iters 10 > gpurun_out/ab/attn_noslp_$r.log 2>&1
done
timeout -k 10 200 python tools/bench_kernels.py --iters 5 --gemm-variants 5 > gpurun_out/ab/k_def.log 2>&1
VP_HIP_LIB=abl/noslp_all/libvp_hip.so timeout -k 10 200 python tools/bench_kernels.py --iters 5 --gemm-variants 5 > gpurun_out/ab/k_noslp_all.log 2>&1
VP_HIP_LIB=abl/noslp_all/libvp_hip.so timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab/bench_noslp_all.log 2>&1
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/ab/bench_def.log 2>&1
