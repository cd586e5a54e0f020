#!/bin/bash
# Sequential bench runs for A/B: each line of $RUNS is "name|ENV=V ...|bench args"; own time limit each,
# the first failure ends the script.  Results: gpurun_out/ab_<name>.json / .err
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
while IFS='|' read -r name envs args; do
  [ -z "$name" ] && continue
  echo "== $name ($envs) $args"
  env $envs timeout -k 10 600 python bench.py $args > "gpurun_out/ab_$name.json" 2> "gpurun_out/ab_$name.err"
  rc=$?
  tail -1 "gpurun_out/ab_$name.err"
  python - "$name" <<'PY'
import json, sys
d = json.load(open(f"gpurun_out/ab_{sys.argv[1]}.json")); e = d["detail"]["engine_per_rank"]; el = d["detail"]["elapsed_s"]
unc = e["prompt_tokens"] - e["cached_tokens"]
print(sys.argv[1], "decisions/s", d["value"], "tok/s %.0f" % ((unc + e["generated_tokens"]) / el),
      "prefill_chunks", e["prefill_chunks"], "rows %.0f" % (e["decode_row_steps"] / max(1, e["decode_steps"])))
PY
  [ $rc -eq 0 ] || { echo "run $name failed rc=$rc"; exit $rc; }
done <<< "$RUNS"
