#!/bin/bash
# rocprofv3 kernel stats of the cascade A/B at the bench geometry (round 3).
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_cascade -o run -- \
  python3 tools/bench_cascade.py --b 608 --shared 40 --group 24 --rounds 2 > gpurun_out/r3_prof_cascade.log 2>&1 \
  || { tail -30 gpurun_out/r3_prof_cascade.log; exit 1; }
tail -3 gpurun_out/r3_prof_cascade.log
f=$(find gpurun_out/prof_cascade -name '*kernel_stats.csv' | head -1)
cut -c1-220 "$f" | head -12
