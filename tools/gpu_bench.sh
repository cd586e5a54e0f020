#!/bin/bash
# GPU tests (optional) + smoke + default bench; each step time-limited, first failure ends it.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
PYT="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
step() {  # name, limit, command...
  local name=$1 limit=$2; shift 2
  echo "== $name"
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -${TAILN:-6} "gpurun_out/$name.log"
  [ $rc -eq 0 ] || { echo "step $name failed rc=$rc"; exit $rc; }
}
[ -z "$TESTS" ] || step gputests 900 $PYT $TESTS -m gpu
echo "== bench"
timeout -k 10 900 python bench.py ${BENCH_ARGS} > gpurun_out/bench${TAG}.json 2> gpurun_out/bench${TAG}.err
rc=$?
tail -3 gpurun_out/bench${TAG}.err
cat gpurun_out/bench${TAG}.json
exit $rc
