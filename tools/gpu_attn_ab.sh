#!/bin/bash
# Attention tests on the in-tree library, prefill A/B of build/libbcg_{base,new}.so, then the driver bench.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "prefill or decode or attention" > gpurun_out/attn_tests.log 2>&1 || { tail -40 gpurun_out/attn_tests.log; exit 1; }
tail -3 gpurun_out/attn_tests.log
VARIANTS="base new" NTS=4 bash tools/gpu_prefill_attn.sh || exit 1
VARIANTS="base new" NTS=4 bash tools/gpu_prefill_attn.sh || exit 1
[ -n "$SKIP_BENCH" ] || { timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; tail -2 gpurun_out/bench.err; cat gpurun_out/bench.json; exit $rc; }
