#!/bin/bash
# rocprofv3 kernel stats of the real-shape TP engine test (Qwen3-32B TP=4 as 4 processes on one GPU):
# which GEMM kernels the TP forward runs (hand gemm_nt with the fused SiLU epilogue).
set -o pipefail
mkdir -p gpurun_out/tp_prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tp_prof -o run -- \
  python -m pytest -x -q --timeout 400 tests/test_tp_real_shapes_gpu.py -k "qwen3-32b-None-4" > gpurun_out/tp_prof/test.log 2>&1
rc=$?
tail -3 gpurun_out/tp_prof/test.log
for f in $(find gpurun_out/tp_prof -name "*kernel_stats.csv"); do echo "== $f"; cut -d, -f1-4 "$f" | head -14 | cut -c1-200; done
find gpurun_out/tp_prof -name "*kernel_trace.csv" -delete
exit $rc
