#!/bin/bash
# Round 3: shipped-GEMM dispatch tests (passed-test output shown: the table entries touched),
# then the driver's bench command and a long (70-window) run of the same pool.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -z "$SKIP_DISPATCH" ]; then
  timeout -k 10 300 python -u -m pytest -x -v -rP --timeout 240 --timeout-method thread tests/test_gemm_dispatch_gpu.py \
    > gpurun_out/dispatch_tests.log 2>&1 || { tail -30 gpurun_out/dispatch_tests.log; exit 1; }
  grep -E "^\[table\]|^\[decoder\]|passed|failed" gpurun_out/dispatch_tests.log | tail -25
fi
echo "== bench (driver command)"
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
if [ -n "$LONG" ]; then
  echo "== long run ($LONG windows)"
  timeout -k 10 900 python bench.py --gpus 1 --steps $LONG --warmup 5 --deadline-s 840 ${BENCH_ARGS} \
    > gpurun_out/bench_long.json 2> gpurun_out/bench_long.err || { tail -20 gpurun_out/bench_long.err; exit 1; }
  cat gpurun_out/bench_long.json
fi
