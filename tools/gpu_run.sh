#!/bin/bash
# The one GPU-box runner (run it through gpurun): every step time-limited, the first failure ends
# the call, logs under gpurun_out/.  Subcommands:
#
#   tools/gpu_run.sh tests [pytest args]        GPU test suite (default: tests -m gpu)
#   tools/gpu_run.sh bench [bench.py args]      headline bench -> gpurun_out/bench/<TAG>.json
#   tools/gpu_run.sh prof  [bench.py args]      rocprofv3 kernel trace + stats of the bench, busy
#                                               windows (trace_overlap.py) and the prefill/decode
#                                               split (phase_split.py) -> gpurun_out/prof/
#   tools/gpu_run.sh pmc KERNEL_FILTER COUNTERS -- CMD...   one rocprofv3 --pmc pass over CMD
#   tools/gpu_run.sh gemm-variants              build/pp_* binaries over $SHAPES (2 interleaved
#                                               rounds, cdna_hip_programming.md rule 24)
#   tools/gpu_run.sh tune MODEL [tune_hand_gemm.py args]   GEMM dispatch table -> gpurun_out/tune/
#   tools/gpu_run.sh tp-rehearsal               real-shape TP tests + TP=2 bench pools on ONE GPU
#
# Env: TAG (file tag), LIMIT (seconds per step), SHAPES / VARIANTS (gemm-variants).
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
cmd=${1:-tests}; shift || true
TAG=${TAG:-run}
mkdir -p gpurun_out

step() {  # name limit command...
  local name=$1 limit=$2; shift 2
  echo "== $name"
  mkdir -p "$(dirname "gpurun_out/$name")"
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -${TAILN:-8} "gpurun_out/$name.log"
  [ $rc -eq 0 ] || { echo "step $name failed rc=$rc"; exit $rc; }
}

case "$cmd" in
  tests)
    [ $# -gt 0 ] || set -- tests -m gpu
    step "tests/$TAG" "${LIMIT:-1100}" python -u -m pytest -x -q --timeout 120 --timeout-method thread "$@"
    ;;
  bench)
    mkdir -p gpurun_out/bench
    timeout -k 10 "${LIMIT:-700}" python -u bench.py "$@" > "gpurun_out/bench/$TAG.json" 2> "gpurun_out/bench/$TAG.err"
    rc=$?
    tail -3 "gpurun_out/bench/$TAG.err"
    cut -c1-900 "gpurun_out/bench/$TAG.json"
    exit $rc
    ;;
  prof)
    cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
    mkdir -p "gpurun_out/prof/$TAG"
    timeout -k 10 "${LIMIT:-900}" rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/prof/$TAG" \
      -o run -- python bench.py "$@" > "gpurun_out/prof/$TAG/bench.json" 2> "gpurun_out/prof/$TAG/bench.err"
    rc=$?
    tail -3 "gpurun_out/prof/$TAG/bench.err"
    cut -c1-600 "gpurun_out/prof/$TAG/bench.json"
    trace=$(find "gpurun_out/prof/$TAG" -name "*kernel_trace.csv" | head -1)
    if [ -n "$trace" ]; then
      python tools/trace_overlap.py "$trace" --window 12 > "gpurun_out/prof/$TAG/busy.json" 2>&1
      python tools/phase_split.py "$trace" --skip-s "${SKIP_S:-150}" > "gpurun_out/prof/$TAG/phase_split.json" 2>&1
      tail -30 "gpurun_out/prof/$TAG/phase_split.json"
      gzip -9 "$trace"
      find "gpurun_out/prof/$TAG" -name "*.gz" -size +40M -delete
    fi
    exit $rc
    ;;
  pmc)
    filter=$1 counters=$2; shift 2; [ "$1" = "--" ] && shift
    cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
    out="gpurun_out/pmc/$TAG"
    mkdir -p "$out"
    timeout -s KILL "${LIMIT:-120}" rocprofv3 --pmc ${counters//,/ } --kernel-include-regex "$filter" \
      --output-format csv -d "$out" -o run -- "$@" > "$out/run.log" 2>&1 || { tail -5 "$out/run.log"; exit 1; }
    python tools/pmc_summary.py "$out" | tee "$out/summary.txt"
    ;;
  gemm-variants)
    SHAPES=${SHAPES:-"16384,34816,5120,1,1 16384,5120,17408,2,1 16384,7168,5120,0,1 16384,5120,5120,2,1"}
    mkdir -p gpurun_out/gemmv
    for round in 1 2; do
      for v in ${VARIANTS:-$(ls build | grep '^pp_' | sed 's/^pp_//')}; do
        for s in $SHAPES; do
          timeout -k 5 60 "build/pp_$v" ${s//,/ } ${ITERS:-20} || { echo "variant $v shape $s failed"; exit 1; }
        done
      done
    done | tee "gpurun_out/gemmv/$TAG.jsonl"
    ;;
  tune)
    model=$1; shift
    mkdir -p gpurun_out/tune
    step "tune/$TAG" "${LIMIT:-900}" python -u tools/tune_hand_gemm.py --model "$model" \
      --out "gpurun_out/tune/$TAG.json" "$@"
    ;;
  tp-rehearsal)
    # Configs 4 and 5 at real shapes on ONE GPU (ranks share cuda:0; gloo + the xGMI all-reduce
    # kernels forced over IPC peer buffers).  Rehearsal only: the ranks time-share one GPU.
    step "tp/tests" "${LIMIT:-600}" python -u -m pytest -x -v -rP --timeout 540 --timeout-method thread \
      tests/test_tp_real_shapes_gpu.py
    COMMON="--one-device --steps ${STEPS:-4} --warmup 1 --fill-max-s 120 --deadline-s 1500"
    step "tp/qwen3_32b_tp2" 600 python bench.py --gpus 2 --tp 2 --model qwen3-32b --sims-per-gpu 16 \
      --max-batch-seqs 160 --kv-cache-gb 12 $COMMON
    step "tp/mistral22b_fp8_tp2" 600 python bench.py --gpus 2 --tp 2 --model mistral-22b --quantization fp8 \
      --honest 16 --byzantine 4 --sims-per-gpu 8 --max-batch-seqs 160 --kv-cache-gb 8 $COMMON
    ;;
  *)
    echo "unknown subcommand $cmd"; exit 2
    ;;
esac
