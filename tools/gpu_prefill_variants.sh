#!/bin/bash
# Prefill attention variant A/B: the in-tree library vs build/libbcg_<v>.so for each v in $VARIANTS
# (tools/bench_prefill.py attention shapes, two alternating rounds).
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  echo "== default"; timeout -k 10 120 python -u tools/bench_prefill.py --skip-gemm 2>&1 | grep attn || exit 1
  for v in $VARIANTS; do
    echo "== $v"; BCG_KERNELS_LIB=$PWD/build/libbcg_$v.so timeout -k 10 120 python -u tools/bench_prefill.py --skip-gemm 2>&1 | grep attn || exit 1
  done
done
