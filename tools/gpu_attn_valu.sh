#!/bin/bash
# Prefill attention / shared-prefix decode with the scores read once (round 3): GPU tests, then
# tools/bench_prefill.py + tools/bench_cascade.py A/B against build/libbcg_silu_old.so (the previous kernels).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_cascade_gpu.py \
  -k "prefill or decode or attention or cascade or shared" > gpurun_out/attn_valu_tests.log 2>&1 || { tail -40 gpurun_out/attn_valu_tests.log; exit 1; }
tail -2 gpurun_out/attn_valu_tests.log
for r in 1 2; do
  echo "== old run $r"
  BCG_KERNELS_LIB=$PWD/build/libbcg_silu_old.so timeout -k 10 120 python -u tools/bench_prefill.py --skip-gemm > gpurun_out/attn_old.log 2>&1 || { tail -5 gpurun_out/attn_old.log; exit 1; }
  grep attn gpurun_out/attn_old.log
  echo "== new run $r"
  timeout -k 10 120 python -u tools/bench_prefill.py --skip-gemm > gpurun_out/attn_new.log 2>&1 || { tail -5 gpurun_out/attn_new.log; exit 1; }
  grep attn gpurun_out/attn_new.log
done
echo "== cascade old"; BCG_KERNELS_LIB=$PWD/build/libbcg_silu_old.so timeout -k 10 200 python -u tools/bench_cascade.py > gpurun_out/casc_old.log 2>&1 || { tail -5 gpurun_out/casc_old.log; exit 1; }
grep -E '"B": 608' gpurun_out/casc_old.log | head -6
echo "== cascade new"; timeout -k 10 200 python -u tools/bench_cascade.py > gpurun_out/casc_new.log 2>&1 || { tail -5 gpurun_out/casc_new.log; exit 1; }
grep -E '"B": 608' gpurun_out/casc_new.log | head -6
