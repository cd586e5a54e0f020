#!/bin/bash
# TP collective fallback rehearsal on ONE GPU (ranks share cuda:0 over gloo; mechanism only):
# the custom all-reduce is cross-checked at init; an injected IPC-mapping failure or result
# mismatch (BCG_AR_FAULT) must make every rank fall back and label config.custom_allreduce.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/tp
run() {  # name limit env... -- bench args
  local name=$1 limit=$2; shift 2
  echo "== $name"
  timeout -k 10 "$limit" env "$@" > "gpurun_out/tp/$name.json" 2> "gpurun_out/tp/$name.err"
  local rc=$?
  python3 - "gpurun_out/tp/$name.json" <<'PY'
import json, sys
lines = [l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")]
d = json.loads(lines[-1]) if lines else {}
print({k: d.get("config", {}).get(k) for k in ("parallelism", "custom_allreduce", "hip_graphs")},
      "decisions", d.get("detail", {}).get("decisions"), "value", d.get("value"))
PY
  [ $rc -eq 0 ] || { echo "step $name failed rc=$rc"; tail -20 "gpurun_out/tp/$name.err"; exit $rc; }
}
TINY="--model bcg/tiny-qwen3 --honest 4 --byzantine 1 --sims-per-gpu 4 --steps 2 --warmup 1 --window-s 6 --fill-max-s 60 --kv-cache-gb 2 --deadline-s 300 --one-device"
run tp2_on 360 BCG_AR_FAULT= python3 bench.py --gpus 2 --tp 2 $TINY &&
run tp2_fault_ipc 360 BCG_AR_FAULT=ipc python3 bench.py --gpus 2 --tp 2 $TINY &&
run tp2_fault_mismatch 360 BCG_AR_FAULT=mismatch python3 bench.py --gpus 2 --tp 2 $TINY &&
run tp4_fault_ipc 560 BCG_AR_FAULT=ipc python3 bench.py --gpus 4 --tp 4 --model qwen3-8b --honest 4 --byzantine 1 \
  --sims-per-gpu 2 --steps 2 --warmup 1 --window-s 20 --fill-max-s 240 --kv-cache-gb 4 --deadline-s 520 --one-device
