#!/bin/bash
# Round-trip on a GPU box: new collective tests, full GPU suite, smoke, default bench.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
step() {  # name, limit, command...
  local name=$1 limit=$2; shift 2
  echo "== $name"
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -25 "gpurun_out/$name.log"
  [ $rc -eq 0 ] || { echo "step $name failed rc=$rc"; exit $rc; }
}
[ -n "$SKIP_AR" ] || step allreduce 240 $PYT tests/test_allreduce.py -m gpu
[ -n "$SKIP_TESTS" ] || step gputests 900 $PYT tests -m gpu
[ -n "$SKIP_SMOKE" ] || step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
if [ -z "$SKIP_BENCH" ]; then
  echo "== bench"
  timeout -k 10 900 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?
  tail -4 gpurun_out/bench.err
  cat gpurun_out/bench.json
  exit $rc
fi
