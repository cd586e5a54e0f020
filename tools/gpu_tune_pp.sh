#!/bin/bash
# Re-tune the decode buckets >= 288 rows and the prefill chunk sizes with the ping-pong kernel
# (cfg 10) against the shipped table's best and the library; merged table -> gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
MODEL=${MODEL:-qwen3-14b}
timeout -k 10 1000 python -u tools/tune_hand_gemm.py --model $MODEL --merge --cfgs 10 --reps ${REPS:-7} \
    --m ${MS:-288,320,352,384,416,448,480,512,544,576,608,640,672,704,736,768,2048,4096,8192,16384} \
    --out gpurun_out/hand_gemm_${MODEL}.json ${EXTRA} > gpurun_out/tune_pp_${MODEL}.log 2>&1
rc=$?
tail -5 gpurun_out/tune_pp_${MODEL}.log
exit $rc
