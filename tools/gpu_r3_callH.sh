#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/tp
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -v -rP --timeout 240 --timeout-method thread tests/test_allreduce.py -m gpu \
  > gpurun_out/tp/ar_tests.log 2>&1 || { grep -E "tp-collectives|FAIL|Error" gpurun_out/tp/ar_tests.log | tail -20; exit 1; }
grep -E "passed|failed" gpurun_out/tp/ar_tests.log | tail -2
SKIP_TESTS=1 bash tools/gpu_tp_rehearsal.sh
