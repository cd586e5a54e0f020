#!/bin/bash
# Full hand-GEMM dispatch table for one model: every decode graph bucket x projection.
set -o pipefail
mkdir -p gpurun_out
MODEL=${MODEL:-qwen3-14b}
M=$(python -c "from byzantine_consensus_llm_agents_amd.engine.graphs import BUCKETS; print(','.join(map(str, BUCKETS)))")
timeout -k 10 900 python -u tools/tune_hand_gemm.py --model $MODEL --m $M --reps ${REPS:-7} \
    --out gpurun_out/hand_gemm_${MODEL}.json ${EXTRA} > gpurun_out/tune_hand_${MODEL}.log 2>&1
rc=$?
tail -5 gpurun_out/tune_hand_${MODEL}.log
exit $rc
