#!/bin/bash
# Ping-pong GEMM: correctness tests, then timing vs hipBLASLt on the Qwen3-14B shapes.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -k "pp or 10" > gpurun_out/pp_test.log 2>&1; rc=$?
tail -5 gpurun_out/pp_test.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/bench_pp.py --m ${MS:-448,768,16384} ${EXTRA} > gpurun_out/pp_bench.log 2>&1; rc=$?
cat gpurun_out/pp_bench.log | tail -30
exit $rc
