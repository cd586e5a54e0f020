#!/bin/bash
# Prefill attention latency ablation (timing only): reloads hit chunk 0's L2-hot blocks vs the real stream.
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  echo "== real"; timeout -k 10 120 python -u tools/bench_prefill.py --skip-gemm 2>&1 | grep attn || exit 1
  echo "== hot";  BCG_KERNELS_LIB=$PWD/build/libbcg_abl_hot.so timeout -k 10 120 python -u tools/bench_prefill.py --skip-gemm 2>&1 | grep attn || exit 1
done
