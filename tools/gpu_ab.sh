#!/bin/bash
# A/B of an engine toggle on the flagship bench: engine GPU tests, then bench with VAR=A and VAR=B.
#   VAR=BCG_OVERLAP_PREFILL A=1 B=0 SIMS=32 bash tools/gpu_ab.sh
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
if [ -z "$NOTEST" ]; then
echo "== engine tests"; timeout -k 10 500 python -m pytest tests/test_engine_gpu.py -x -q > gpurun_out/engine_tests.log 2>&1; rc=$?; tail -5 gpurun_out/engine_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for val in $A $B; do
echo "== bench $VAR=$val"
env $VAR=$val timeout -k 10 900 python bench.py --steps ${STEPS:-2} --warmup 1 --sims-per-gpu ${SIMS:-32} > gpurun_out/bench_$val.json 2> gpurun_out/bench_$val.err; rc=$?
tail -2 gpurun_out/bench_$val.err; cat gpurun_out/bench_$val.json; [ $rc -eq 0 ] || exit $rc
done
