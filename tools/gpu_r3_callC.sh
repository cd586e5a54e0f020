#!/bin/bash
# The driver's bench command at the current defaults, then a rocprofv3 kernel trace of the same bench (tools/gpu_r3_prof.sh).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err \
  || { tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
SKIP_FP8=1 STEPS=${PROF_STEPS:-10} bash tools/gpu_r3_prof.sh
