#!/bin/bash
# glds-ring prefill attention (nt = 8): GPU tests, then timing vs the register kernel (nt = 4)
# at the default head group and at BCG_PREFILL_GT = 3 / 4.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "prefill" > gpurun_out/prefill_tests.log 2>&1 || { tail -40 gpurun_out/prefill_tests.log; exit 1; }
tail -2 gpurun_out/prefill_tests.log
for gt in 0 3 4; do
  BCG_PREFILL_GT=$gt timeout -k 10 120 python -u tools/bench_prefill.py --skip-gemm --nts 4,8 \
    > gpurun_out/prefill_dma_gt$gt.log 2>&1 || { tail -5 gpurun_out/prefill_dma_gt$gt.log; exit 1; }
  echo "== GT=$gt"; grep attn gpurun_out/prefill_dma_gt$gt.log
done
