#!/bin/bash
# Kernel-level profile of a short bench run (rocprofv3 kernel trace + stats).
set -o pipefail
mkdir -p gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python bench.py --steps ${STEPS:-6} --warmup ${WARMUP:-4} --sims-per-gpu ${SIMS:-128} ${EXTRA} > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err
rc=$?
tail -3 gpurun_out/prof_bench.err
cat gpurun_out/prof_bench.json
# keep the summaries; the full per-dispatch trace is too large to ship back
find gpurun_out/prof -name "*kernel_trace*" -exec gzip -9 {} \;
find gpurun_out/prof -name "*.gz" -size +40M -delete
find gpurun_out/prof -name "*stats*" | head
exit $rc
