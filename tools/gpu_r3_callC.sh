#!/bin/bash
# fp8 256x256 kernel (tests + prefill shapes vs _scaled_mm), the driver's bench command at the
# current defaults, then a rocprofv3 kernel trace of the same bench (tools/gpu_r3_prof.sh).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -m gpu \
  -k "pp" > gpurun_out/pp_tests.log 2>&1 || { tail -30 gpurun_out/pp_tests.log; exit 1; }
tail -1 gpurun_out/pp_tests.log
timeout -k 10 300 python -u tools/bench_fp8_gemm.py --ms 8192,16384 > gpurun_out/fp8_prefill.log 2>&1 \
  || { tail -20 gpurun_out/fp8_prefill.log; exit 1; }
cat gpurun_out/fp8_prefill.log
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err \
  || { tail -20 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
SKIP_FP8=1 STEPS=${PROF_STEPS:-10} bash tools/gpu_r3_prof.sh
