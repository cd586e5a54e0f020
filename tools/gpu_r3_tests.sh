#!/bin/bash
# Full GPU suite + smoke at HEAD (round 3 close-out).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/head_gputests.log 2>&1 \
  || { tail -40 gpurun_out/head_gputests.log; exit 1; }
tail -2 gpurun_out/head_gputests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/head_smoke.log 2>&1 || { tail -20 gpurun_out/head_smoke.log; exit 1; }
tail -2 gpurun_out/head_smoke.log
