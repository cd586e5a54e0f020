#!/bin/bash
# Kernel-level profile of the headline bench at the current defaults (round 3, re-entry):
# rocprofv3 kernel trace + stats, GPU idle per 8-s window, and the prefill / decode split of
# kernel time per kernel family (tools/phase_split.py, start-up skipped).
set -o pipefail
mkdir -p gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python bench.py --steps ${STEPS:-10} --warmup ${WARMUP:-5} ${EXTRA} > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err
rc=$?
tail -3 gpurun_out/prof_bench.err
cat gpurun_out/prof_bench.json
tr=$(find gpurun_out/prof -name "*kernel_trace.csv" | head -1)
python tools/trace_overlap.py "$tr" --window 8 > gpurun_out/prof/busy.json 2>&1
tail -3 gpurun_out/prof/busy.json
python tools/phase_split.py "$tr" --skip-s ${SKIP_S:-150} > gpurun_out/prof/phase_split.json 2>&1
cat gpurun_out/prof/phase_split.json
find gpurun_out/prof -name "*kernel_trace*" -exec gzip -9 {} \;
find gpurun_out/prof -name "*.gz" -size +40M -delete
exit $rc
