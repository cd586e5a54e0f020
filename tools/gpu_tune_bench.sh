#!/bin/bash
# Extend the shipped TunableOp table to every decode bucket, install it, then bench.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
MODEL=${MODEL:-qwen3-14b}
NAME=${NAME:-qwen3-14b}
TBL=byzantine_consensus_llm_agents_amd/engine/tuned/tunableop_${NAME}_tp1.csv
echo "== tune"
timeout -k 10 900 python tools/tune_gemms.py --model $MODEL --max-m 768 --base $TBL \
  --out gpurun_out/tunableop_${NAME}_tp1.csv > gpurun_out/tune.log 2>&1 || { tail -20 gpurun_out/tune.log; exit 1; }
tail -3 gpurun_out/tune.log
cp gpurun_out/tunableop_${NAME}_tp1.csv $TBL
if [ -z "$SKIP_BENCH" ]; then
  echo "== bench"
  timeout -k 10 900 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; tail -3 gpurun_out/bench.err; cat gpurun_out/bench.json; exit $rc
fi
