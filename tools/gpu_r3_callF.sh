#!/bin/bash
# 256x256 tile-order (GROUP_M) variants on the prefill shapes, then the TP = 2 engine rehearsal.
set -o pipefail
SKIP_TESTS=1 SHAPES="16384,34816,5120,1,1 16384,5120,17408,2,1 16384,7168,5120,0,1 16384,5120,5120,2,1 9000,7168,5120,0,1 9000,5120,17408,2,1" \
  timeout -k 10 400 bash tools/gpu_gemm_variants.sh > gpurun_out/gemmv_groupm.log 2>&1 || { tail -20 gpurun_out/gemmv_groupm.log; exit 1; }
python tools/gemm_variant_table.py gpurun_out/gemmv/times.jsonl > gpurun_out/gemmv/table.txt 2>&1; cat gpurun_out/gemmv/table.txt
SKIP_TESTS=1 bash tools/gpu_tp_rehearsal.sh
