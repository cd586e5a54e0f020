#!/bin/bash
# Decode-attention tests + op timing, then the batch-cap sweep; every GPU step time-limited.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "decode" > gpurun_out/attn_tests.log 2>&1 || { tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -3 gpurun_out/attn_tests.log
timeout -k 10 300 python tools/bench_ops.py --skip-gemm --ms 160,448,608,768 --ctx 900 > gpurun_out/ops_ctx900.log 2>&1 \
  || { tail -20 gpurun_out/ops_ctx900.log; exit 1; }
grep -i "attn\|attention" gpurun_out/ops_ctx900.log | head -20
bash tools/gpu_batch_sweep.sh
