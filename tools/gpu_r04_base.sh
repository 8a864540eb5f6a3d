#!/bin/bash
# round 4, first GPU call: the measurements VERDICT r03 asked for before any new variant
#   p2 attention PMC (3 passes) + GEMM PMC (2 passes), the fp8 DMA A/B, the config-5 full-model test on HEAD,
#   config 4 / 5 bench lines with rocprof kernel stats
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local name=$1; shift; local to=$1; shift
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "$name rc=$rc"
  [ $rc -ne 0 ] && { tail -20 "gpurun_out/$name.log"; exit $rc; }; return 0; }
run r04_c5_model_test 400 python -u -m pytest tests/test_model_gpu.py -k config5 -x -v -s --timeout 360 --timeout-method thread
run r04_f8_tests 300 python -u -m pytest tests/test_attention_fp8_gpu.py -x -q --timeout 120 --timeout-method thread
: > gpurun_out/r04_f8dma_ab.log
for i in 1 2 3; do
  for L in libvp_hip_f8old.so libvp_hip.so; do
    echo "== $L" >> gpurun_out/r04_f8dma_ab.log
    VP_HIP_LIB=$PWD/videopainter_amd/_lib/$L timeout -k 10 120 python tools/bench_kernels.py --only attn8 --variant8 3 --video-tokens 46800 --iters 10 2>&1 | grep "attention fp8" >> gpurun_out/r04_f8dma_ab.log || exit 1
  done
done
cat gpurun_out/r04_f8dma_ab.log
bash tools/pmc_attn_p1.sh p2 || exit 1
bash tools/pmc_gemm.sh 11 || exit 1
rm -rf gpurun_out/r04_c5_prof gpurun_out/r04_c4_prof
run r04_bench_c5 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_c5_prof -o k --output-format csv -- python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline
run r04_bench_c4 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_c4_prof -o k --output-format csv -- python bench.py --config 4 --steps 2 --warmup 1
exit 0
