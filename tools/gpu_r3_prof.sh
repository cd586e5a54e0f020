#!/bin/bash
# fp8 prefill GEMMs (hand 256x256 fp8 vs _scaled_mm), then a kernel-level profile of the
# headline bench (age-mixed pool, steady state): rocprofv3 kernel trace + stats.
set -o pipefail
mkdir -p gpurun_out/prof
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -z "$SKIP_FP8" ]; then
  timeout -k 10 400 python -u tools/bench_fp8_gemm.py --ms ${FP8_MS:-2048,8192,16384} > gpurun_out/fp8_prefill.log 2>&1 \
    || { tail -20 gpurun_out/fp8_prefill.log; exit 1; }
  cat gpurun_out/fp8_prefill.log
fi
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
  python bench.py --steps ${STEPS:-10} --warmup ${WARMUP:-5} ${EXTRA} > gpurun_out/prof_bench.json 2> gpurun_out/prof_bench.err
rc=$?
tail -3 gpurun_out/prof_bench.err
cat gpurun_out/prof_bench.json
python tools/trace_overlap.py $(find gpurun_out/prof -name "*kernel_trace.csv" | head -1) --window 8 > gpurun_out/prof/busy.json 2>&1
tail -3 gpurun_out/prof/busy.json
find gpurun_out/prof -name "*kernel_trace*" -exec gzip -9 {} \;
find gpurun_out/prof -name "*.gz" -size +40M -delete
exit $rc
