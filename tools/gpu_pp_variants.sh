#!/bin/bash
# Time every build/pp_* variant on the decode / prefill shapes, then PMC passes over one variant.
set -o pipefail
mkdir -p gpurun_out/ppv
export HSA_ENABLE_IPC_MODE_LEGACY=0
SHAPES=${SHAPES:-"16384,34816,5120,1,1 16384,5120,17408,2,1 768,34816,5120,1,1 768,5120,17408,2,4 768,151936,5120,0,1 768,7168,5120,0,3"}
for v in ${VARIANTS:-$(ls build | grep '^pp_' | sed 's/^pp_//')}; do
  for s in $SHAPES; do
    timeout -k 5 60 build/pp_$v ${s//,/ } 30 || { echo "variant $v shape $s failed"; exit 1; }
  done
done | tee gpurun_out/ppv/times.jsonl
[ -z "$PMC_VARIANTS" ] && exit 0
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
GROUPS_TXT=${PMC_GROUPS:-"SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_INSTS_MFMA,SQ_VALU_MFMA_BUSY_CYCLES;SQ_INSTS_LDS,SQ_LDS_BANK_CONFLICT,SQ_ACTIVE_INST_LDS,SQ_WAIT_INST_LDS,SQ_INST_CYCLES_VMEM,GRBM_GUI_ACTIVE;FETCH_SIZE,TCC_HIT_sum;TCC_HIT_sum,TCC_MISS_sum,GRBM_GUI_ACTIVE"}
for v in $PMC_VARIANTS; do
  i=0
  IFS=';' read -ra GROUPS_ARR <<< "$GROUPS_TXT"
  for group in "${GROUPS_ARR[@]}"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc ${group//,/ } --output-format csv -d gpurun_out/ppv/$v/p$i -o run -- \
      build/pp_$v ${PMC_SHAPE//,/ } 10 > gpurun_out/ppv/$v.p$i.log 2>&1 || { echo "pass $v/$i failed: $group"; tail -3 gpurun_out/ppv/$v.p$i.log; exit 1; }
    echo "pass $v/$i ok: $group"
  done
  echo "== $v"; python tools/pmc_summary.py gpurun_out/ppv/$v | grep -A40 "gemm_" | tee gpurun_out/ppv/summary_$v.txt
done
