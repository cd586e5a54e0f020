#!/bin/bash
# Configs 4 and 5 at real shapes on ONE GPU (ranks share cuda:0; gloo + the xGMI all-reduce kernels
# forced over IPC peer buffers): the real-shape TP numerics tests (TP = 4 on gloo collectives,
# TP = 2 on the xGMI kernels), then the bench pool through the TP = 2 engine (driver/follower
# plans, decode graphs with the all-reduce inside; prefill chunks above the kernel cap
# go through the xGMI kernels in pieces, not gloo host copies: TPGroup.chunk_large).  The plan-exchange cost is in
# detail.phases_rank0 (plan_exchange).  Rehearsal only: the ranks time-share one GPU, so the
# decisions/s here are not a measurement.  (TP = 4 engine runs need 4 co-resident ranks: only on
# a node with one GPU per rank, see tests/test_tp_real_shapes_gpu.py.)
set -o pipefail
mkdir -p gpurun_out/tp
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -v -rP --timeout 540 --timeout-method thread tests/test_tp_real_shapes_gpu.py \
    > gpurun_out/tp/tests.log 2>&1 || { tail -40 gpurun_out/tp/tests.log; exit 1; }
  grep -E "tp-real|passed|failed" gpurun_out/tp/tests.log | tail -5
fi
COMMON="--one-device --steps ${STEPS:-4} --warmup 1 --fill-max-s 120 --deadline-s 1500"
echo "== Qwen3-32B TP=2, 8h+2b"
timeout -k 10 600 python bench.py --gpus 2 --tp 2 --model qwen3-32b --sims-per-gpu 16 --max-batch-seqs 160 \
  --kv-cache-gb 12 $COMMON > gpurun_out/tp/tp2_qwen3_32b.json 2> gpurun_out/tp/tp2_qwen3_32b.err \
  || { tail -30 gpurun_out/tp/tp2_qwen3_32b.err; exit 1; }
cat gpurun_out/tp/tp2_qwen3_32b.json
echo "== Mistral-22B fp8 TP=2, 16h+4b"
timeout -k 10 600 python bench.py --gpus 2 --tp 2 --model mistral-22b --quantization fp8 --honest 16 --byzantine 4 \
  --sims-per-gpu 8 --max-batch-seqs 160 --kv-cache-gb 8 $COMMON > gpurun_out/tp/tp2_mistral22b_fp8.json \
  2> gpurun_out/tp/tp2_mistral22b_fp8.err || { tail -30 gpurun_out/tp/tp2_mistral22b_fp8.err; exit 1; }
cat gpurun_out/tp/tp2_mistral22b_fp8.json
