#!/bin/bash
# Hand-GEMM dispatch entries for the other BASELINE models' decode shapes (merged later into
# engine/tuned/hand_gemm.json): Qwen3-8B TP=1 (config 2) and Qwen3-32B TP=4 (config 4).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
MS=${MS:-16,32,64,128,192,256,320,384,448,512,576,640,704,768}
for spec in ${SPECS:-qwen3-8b:1 qwen3-32b:4}; do
  model=${spec%%:*}; tp=${spec##*:}
  echo "== $model tp=$tp"
  timeout -k 10 600 python -u tools/tune_hand_gemm.py --model $model --tp $tp --m $MS --reps ${REPS:-7} \
    --out gpurun_out/hand_gemm_${model}_tp$tp.json > gpurun_out/tune_hand_${model}_tp$tp.log 2>&1 \
    || { tail -20 gpurun_out/tune_hand_${model}_tp$tp.log; exit 1; }
  tail -3 gpurun_out/tune_hand_${model}_tp$tp.log
done
