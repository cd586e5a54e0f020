#!/bin/bash
# BASELINE.json configs on ONE MI355X (TP configs run at TP=1 here: the 8-GPU node is the driver's).
#   CONFIGS="c1 c2" bash tools/gpu_configs.sh
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # tag, limit, bench args...
  local tag=$1 limit=$2; shift 2
  echo "== $tag: $*"
  timeout -k 10 "$limit" python bench.py "$@" > gpurun_out/cfg_$tag.json 2> gpurun_out/cfg_$tag.err
  local rc=$?
  tail -2 gpurun_out/cfg_$tag.err; cat gpurun_out/cfg_$tag.json
  [ $rc -eq 0 ] || { echo "config $tag failed rc=$rc"; exit $rc; }
}
for c in ${CONFIGS:-c1 c2}; do
  case $c in
    c1) run c1 300 --model qwen2.5-0.5b --honest 4 --byzantine 0 --max-rounds 5 --sims-per-gpu 64 --steps 3 --warmup 1 ;;
    c2) run c2 600 --model qwen3-8b --honest 8 --byzantine 0 --sims-per-gpu 96 --steps 2 --warmup 1 ;;
    c4) run c4 900 --model qwen3-32b --honest 8 --byzantine 2 --sims-per-gpu 48 --steps 2 --warmup 1 ;;
    c5) run c5 900 --model mistral-22b --quantization fp8 --honest 16 --byzantine 4 --sims-per-gpu 32 --steps 2 --warmup 1 ;;
  esac
done
