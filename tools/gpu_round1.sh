#!/bin/bash
# First GPU validation: kernel tests, engine tests, smoke, short bench.
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
echo "== build"; timeout -k 10 300 python __graft_entry__.py > gpurun_out/build.log 2>&1 || { echo build failed; cat gpurun_out/build.log; exit 1; }
echo "== kernel tests"; timeout -k 10 400 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/kernels.log 2>&1; rc=$?; tail -30 gpurun_out/kernels.log; [ $rc -eq 0 ] || exit $rc
echo "== engine tests"; timeout -k 10 400 python -m pytest tests/test_engine_gpu.py -x -q > gpurun_out/engine.log 2>&1; rc=$?; tail -30 gpurun_out/engine.log; [ $rc -eq 0 ] || exit $rc
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -5 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 900 python bench.py --steps 2 --warmup 1 --sims-per-gpu ${SIMS:-4} --verbose > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; tail -5 gpurun_out/bench.err; cat gpurun_out/bench.json; exit $rc
