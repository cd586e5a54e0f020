#!/bin/bash
# PMC counters of the attention kernels (prefill micro-benchmark + decode micro-benchmark),
# one rocprofv3 pass per counter group, each under its own hard time limit.
set -o pipefail
OUT=${OUT:-gpurun_out/pmc_attn}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $group --output-format csv -d $OUT/p$i -o run -- \
    python tools/bench_prefill.py --skip-gemm > $OUT/p$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i failed rc=$rc: $group"; grep -i -m3 "error" $OUT/p$i.log; exit 1; fi
  echo "pass $i ok: $group"
done <<GROUPS
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_WAIT_INST_LDS
FETCH_SIZE
GROUPS
python tools/pmc_summary.py $OUT > $OUT/summary.txt && grep -A20 prefill_attn $OUT/summary.txt
