#!/bin/bash
# training-gradient accuracy per attention variant (the branch-gradient test prints rel errors), then the LoRA tests
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
T=tests/test_training_gpu.py::test_branch_gradients_through_frozen_transformer
for vu in p2a:p2a w64f:a16 p2:lazy s16:a16; do
  v=${vu%%:*}; u=${vu##*:}
  VP_ATTN_BOUNDED_MODE=$v VP_ATTN_UNBOUNDED_MODE=$u timeout -k 10 200 python -u -m pytest $T -q -s --timeout 120 --timeout-method thread > gpurun_out/r04_train_ab_${v}_$u.log 2>&1
  rc=$?; echo "$v/$u rc=$rc"; grep -E "time_embedding.linear_1|output " gpurun_out/r04_train_ab_${v}_$u.log
  [ $rc -gt 1 ] && exit $rc
done
timeout -k 10 600 python -u -m pytest tests/test_training_gpu.py tests/test_model_gpu.py tests/test_ulysses_gpu.py tests/test_pipeline_contract_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/r04_lora_tests.log 2>&1
rc=$?; echo "lora rc=$rc"; grep -E "FAILED|passed|failed" gpurun_out/r04_lora_tests.log | tail -15
exit 0
