#!/bin/bash
# PMC passes over one GEMM configuration (tools/gemm_probe.py); one rocprofv3 run per counter group.
set -o pipefail
mkdir -p gpurun_out/pmcg
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ARGS=${ARGS:-"--m 768 --n 34816 --k 5120 --epi 1 --cfg 8"}
timeout -k 10 60 python tools/gemm_probe.py $ARGS 2>&1 | grep -v amdgpu.ids
timeout -k 10 60 python tools/gemm_probe.py $ARGS --lib 2>&1 | grep -v amdgpu.ids
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmcg/avail.txt 2>&1 || true
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $group --output-format csv -d gpurun_out/pmcg/p$i -o run -- \
    python tools/gemm_probe.py $ARGS > gpurun_out/pmcg/p$i.log 2>&1 || { echo "pass $i failed: $group"; tail -3 gpurun_out/pmcg/p$i.log; exit 1; }
  echo "pass $i ok: $group"
done <<GROUPS
${PMC_GROUPS:-FETCH_SIZE
TCC_HIT_sum TCC_MISS_sum
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS
TA_BUSY_avr TA_BUSY_max
SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM}
GROUPS
python - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/pmcg/p*/**/*counter_collection*.csv", recursive=True)):
    for row in csv.DictReader(open(f)):
        if "gemm_nt_kernel" not in row.get("Kernel_Name", ""):
            continue
        agg[row["Counter_Name"]].append(float(row["Counter_Value"]))
with open("gpurun_out/pmcg/summary.txt", "w") as out:
    for k, v in sorted(agg.items()):
        line = f"{k:32s} per-dispatch mean {sum(v)/len(v):.4g}  (n={len(v)})"
        print(line); out.write(line + "\n")
PY
