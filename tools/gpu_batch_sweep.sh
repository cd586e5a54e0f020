#!/bin/bash
# Decode batch-cap / pool-size sweep: one bench per "SIMS:CAP" entry of $CONFIGS,
# each under its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for c in ${CONFIGS:-"160:1024 192:1024"}; do
  sims=${c%%:*}; cap=${c##*:}
  echo "== sims=$sims cap=$cap"
  timeout -k 10 600 python bench.py --sims-per-gpu "$sims" --max-batch-seqs "$cap" ${BENCH_ARGS} \
    > "gpurun_out/sweep_s${sims}_c${cap}.json" 2> "gpurun_out/sweep_s${sims}_c${cap}.err"
  rc=$?
  tail -2 "gpurun_out/sweep_s${sims}_c${cap}.err"
  cat "gpurun_out/sweep_s${sims}_c${cap}.json"
  [ $rc -eq 0 ] || { echo "config $c failed rc=$rc"; exit $rc; }
done
