#!/bin/bash
# GPU tests, then the driver's bench command with and without prefill overlapped on a second
# stream (no stream-K library GEMM under overlap: ops/gemm_plan.py avoid_library).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread $TESTS -m gpu > gpurun_out/gputests.log 2>&1 || { tail -20 gpurun_out/gputests.log; exit 1; }
  tail -2 gpurun_out/gputests.log
fi
for ov in ${OVERLAPS:-0 1}; do
  echo "== overlap=$ov"
  BCG_OVERLAP_PREFILL=$ov timeout -k 10 600 python bench.py --gpus 1 --steps ${STEPS:-20} --warmup ${WARMUP:-5} \
      > gpurun_out/bench_ov$ov.json 2> gpurun_out/bench_ov$ov.err || { tail -20 gpurun_out/bench_ov$ov.err; exit 1; }
  tail -c 400 gpurun_out/bench_ov$ov.json | head -c 400; echo
done
