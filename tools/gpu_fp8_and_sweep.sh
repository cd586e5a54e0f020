#!/bin/bash
# fp8 hand-GEMM + large-batch decode-attention tests, fp8 GEMM timing, then a pool-size sweep.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_gpu.py \
  tests/test_kernels_gpu.py -m gpu -k "fp8 or decode" > gpurun_out/fp8_tests.log 2>&1 \
  || { tail -40 gpurun_out/fp8_tests.log; exit 1; }
tail -3 gpurun_out/fp8_tests.log
timeout -k 10 300 python tools/bench_fp8_gemm.py > gpurun_out/bench_fp8_gemm.log 2>&1 \
  || { tail -20 gpurun_out/bench_fp8_gemm.log; exit 1; }
grep "M=" gpurun_out/bench_fp8_gemm.log
[ -z "$CONFIGS" ] || bash tools/gpu_batch_sweep.sh
