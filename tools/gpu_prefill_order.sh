#!/bin/bash
# Prefill attention grid order A/B (round 3): GPU tests with the XCD-aware order, then
# tools/bench_prefill.py attention shapes alternating default / XCD-aware order.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
BCG_PREFILL_XCD_ORDER=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_kernels_gpu.py -k "prefill" > gpurun_out/prefill_order_tests.log 2>&1 || { tail -30 gpurun_out/prefill_order_tests.log; exit 1; }
tail -2 gpurun_out/prefill_order_tests.log
for r in 1 2; do
  for o in 0 1; do
    BCG_PREFILL_XCD_ORDER=$o timeout -k 10 120 python -u tools/bench_prefill.py --skip-gemm > gpurun_out/prefill_order_$o.log 2>&1 \
      || { tail -5 gpurun_out/prefill_order_$o.log; exit 1; }
    echo "order=$o run=$r"; grep attn gpurun_out/prefill_order_$o.log
  done
done
