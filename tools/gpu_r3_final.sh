#!/bin/bash
# Round-3 final check: full GPU suite, smoke, silu A/B, then the driver's bench command.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/final_gputests.log 2>&1 \
  || { tail -40 gpurun_out/final_gputests.log; exit 1; }
tail -2 gpurun_out/final_gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -3 gpurun_out/final_smoke.log
bash tools/gpu_silu_ab.sh > gpurun_out/final_silu_ab.log 2>&1 || { tail -10 gpurun_out/final_silu_ab.log; exit 1; }
cat gpurun_out/final_silu_ab.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || { tail -20 gpurun_out/final_bench.err; exit 1; }
cat gpurun_out/final_bench.json
