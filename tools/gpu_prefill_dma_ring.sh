#!/bin/bash
# glds-ring prefill attention: tests on the in-tree library, then ring depth x head-group timing.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "prefill" > gpurun_out/prefill_tests.log 2>&1 || { tail -40 gpurun_out/prefill_tests.log; exit 1; }
tail -2 gpurun_out/prefill_tests.log
for v in ring3 ring5; do
  for gt in 3 5; do
    BCG_KERNELS_LIB=$PWD/build/libbcg_$v.so BCG_PREFILL_GT=$gt timeout -k 10 120 python -u tools/bench_prefill.py \
      --skip-gemm --nts 8 > gpurun_out/prefill_${v}_gt$gt.log 2>&1 || { tail -5 gpurun_out/prefill_${v}_gt$gt.log; exit 1; }
    echo "== $v GT=$gt"; grep attn gpurun_out/prefill_${v}_gt$gt.log
  done
done
