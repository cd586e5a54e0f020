#!/bin/bash
# Cascade decode attention: GPU tests + kernel A/B (round 3).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_cascade_gpu.py \
  "tests/test_kernels_gpu.py::test_paged_attention_decode" > gpurun_out/r3_cascade_tests.log 2>&1 || { tail -40 gpurun_out/r3_cascade_tests.log; exit 1; }
tail -3 gpurun_out/r3_cascade_tests.log
timeout -k 10 300 python -u tools/bench_cascade.py > gpurun_out/r3_bench_cascade.log 2>&1 || { tail -30 gpurun_out/r3_bench_cascade.log; exit 1; }
cat gpurun_out/r3_bench_cascade.log
