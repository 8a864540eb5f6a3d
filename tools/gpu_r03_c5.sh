#!/bin/bash
# config-5 full-model golden test, then the w64 / w64f attention A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py -x -v -s -m gpu -k "config5_full_model" --timeout 360 \
  --timeout-method thread > gpurun_out/c5_test.log 2>&1
rc=$?; grep -E "config 5 full|PASS|FAIL|passed|failed|Error" gpurun_out/c5_test.log | head; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_r03_w64f2.sh
