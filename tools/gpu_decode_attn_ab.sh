#!/bin/bash
# Decode-attention tests on the in-tree library, then A/B of build/libbcg_{base,new}.so (tools/bench_ops.py).
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -m gpu \
  -k "decode or rope" > gpurun_out/dec_tests.log 2>&1 || { tail -40 gpurun_out/dec_tests.log; exit 1; }
tail -2 gpurun_out/dec_tests.log
for pass in 1 2; do
  for v in base new; do
    for ctx in 900 1700; do
      BCG_KERNELS_LIB=$PWD/build/libbcg_$v.so BCG_BENCH_B=160,448,608,768 timeout -k 10 120 \
        python tools/bench_ops.py --skip-gemm --ctx $ctx > gpurun_out/dec_ab_${v}_$ctx.log 2>&1 \
        || { tail -5 gpurun_out/dec_ab_${v}_$ctx.log; exit 1; }
      echo "$v ctx=$ctx: $(grep '"TBps"' gpurun_out/dec_ab_${v}_$ctx.log | python -c 'import sys,json; print(" ".join(("B%d %.2f" % (d["B"], d["TBps"])) if "B" in d else ("rope T%d %.1fus" % (d["T"], d["rope_us"])) for d in map(json.loads, sys.stdin)))')"
    done
  done
done
