#!/bin/bash
# round 3: the VideoPainterID training backward (resample processor + trainable LoRA factors)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_training_gpu.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/r03_train_tests.log 2>&1
rc=$?; echo "train tests rc=$rc"; exit $rc
