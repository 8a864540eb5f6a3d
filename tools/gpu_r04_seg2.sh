#!/bin/bash
# segment-2 fast DMA path (resample processor): tests, then config-4 bench lines alternating the k2 / v2 layout
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 300 --timeout-method thread -k "k2 or resample or segment or l_extra or null or config4 or fast_path" > gpurun_out/r04_seg2_tests.log 2>&1 || { tail -30 gpurun_out/r04_seg2_tests.log; exit 1; }
tail -1 gpurun_out/r04_seg2_tests.log
: > gpurun_out/r04_seg2_ab.log
for S in 0 1 0 1; do
  VP_RESAMPLE_K2_STRIDED=$S timeout -k 10 300 python bench.py --config 4 --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null | grep "^{" | cut -c1-220 | sed "s/^/strided=$S /" >> gpurun_out/r04_seg2_ab.log || exit 1
done
cat gpurun_out/r04_seg2_ab.log
exit 0
