#!/bin/bash
# Round 3 GEMM A/B: GPU tests of the 256x256 kernels, then every build/pp_* variant on the
# Qwen3-14B prefill / decode shapes (interleaved rounds in one call, rule 24).
set -o pipefail
mkdir -p gpurun_out/gemmv
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py \
    > gpurun_out/gemmv/tests.log 2>&1 || { tail -30 gpurun_out/gemmv/tests.log; exit 1; }
  tail -2 gpurun_out/gemmv/tests.log
fi
SHAPES=${SHAPES:-"16384,34816,5120,1,1 16384,5120,17408,2,1 16384,7168,5120,0,1 16384,5120,5120,2,1 8192,34816,5120,1,1 768,34816,5120,1,1 768,7168,5120,0,3 768,5120,17408,2,4"}
for round in 1 2; do
  for v in ${VARIANTS:-$(ls build | grep '^pp_' | sed 's/^pp_//')}; do
    for s in $SHAPES; do
      timeout -k 5 60 build/pp_$v ${s//,/ } 20 || { echo "variant $v shape $s failed"; exit 1; }
    done
  done
done | tee gpurun_out/gemmv/times.jsonl
