#!/bin/bash
# Iteration loop: kernel tests -> op microbench -> short bench.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "== kernel tests"; timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q > gpurun_out/kernels.log 2>&1; rc=$?; tail -15 gpurun_out/kernels.log; [ $rc -eq 0 ] || exit $rc
echo "== ops"; timeout -k 10 300 python tools/bench_ops.py > gpurun_out/ops.log 2>&1; rc=$?; cat gpurun_out/ops.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
if [ -n "$BENCH" ]; then
echo "== bench"; timeout -k 10 900 python bench.py --steps ${STEPS:-2} --warmup 1 --sims-per-gpu ${SIMS:-16} > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; tail -4 gpurun_out/bench.err; cat gpurun_out/bench.json; exit $rc
fi
