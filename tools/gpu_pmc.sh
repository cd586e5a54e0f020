#!/bin/bash
# PMC counters of the decode-attention microbenchmark (one rocprofv3 pass per counter group).
#   BCG_BENCH_B=160 BCG_ATTN_VARIANTS=1 bash tools/gpu_pmc.sh
set -o pipefail
mkdir -p gpurun_out/pmc
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/bench_ops.py --skip-gemm > gpurun_out/pmc/ops.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/pmc/ops.log
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $group --output-format csv -d gpurun_out/pmc/p$i -o run -- \
    python tools/bench_ops.py --skip-gemm > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; exit 1; }
  echo "pass $i ok: $group"
done <<GROUPS
${PMC_GROUPS:-TA_BUSY_avr TA_BUSY_max
FETCH_SIZE
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
MeanOccupancyPerActiveCU
MemUnitStalled
TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum}
GROUPS
python tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt && cat gpurun_out/pmc/summary.txt
