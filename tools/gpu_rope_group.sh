#!/bin/bash
# rope / KV-write GPU tests (incl. the grouped prefill V writer), then op timing.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  tests/test_engine_gpu.py -m gpu > gpurun_out/rope_tests.log 2>&1 || { tail -40 gpurun_out/rope_tests.log; exit 1; }
tail -2 gpurun_out/rope_tests.log
BCG_BENCH_B=160 timeout -k 10 120 python tools/bench_ops.py --skip-gemm --ctx 900 > gpurun_out/rope_ops.log 2>&1 \
  || { tail -5 gpurun_out/rope_ops.log; exit 1; }
grep rope_us gpurun_out/rope_ops.log
