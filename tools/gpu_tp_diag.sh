#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/tp
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -v -rP --timeout 240 --timeout-method thread tests/test_allreduce.py -m gpu \
  > gpurun_out/tp/ar_tests.log 2>&1; rc=$?
grep -E "tp-collectives|PASS|FAIL|passed|failed" gpurun_out/tp/ar_tests.log | tail -12
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest -v -rP --timeout 280 --timeout-method thread tests/test_tp_real_shapes_gpu.py \
  > gpurun_out/tp/tests.log 2>&1; rc=$?
grep -E "tp-real|PASS|FAIL|passed|failed|Error" gpurun_out/tp/tests.log | tail -12
exit $rc
