#!/bin/bash
# Prefill attention A/B: every build/libbcg_<variant>.so x kernel form (nt), tools/bench_prefill.py shapes.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in ${VARIANTS:-$(ls build | grep '^libbcg_' | sed 's/^libbcg_//; s/\.so$//')}; do
  echo "== $v"
  BCG_KERNELS_LIB=$PWD/build/libbcg_$v.so timeout -k 10 120 python -u tools/bench_prefill.py --skip-gemm \
      > gpurun_out/prefill_attn_$v.log 2>&1 || { tail -5 gpurun_out/prefill_attn_$v.log; exit 1; }
  grep attn gpurun_out/prefill_attn_$v.log
done
