#!/bin/bash
# Prefill attention with the shared K/V ring (BCG_PREFILL_LDS=1): GPU tests, then A/B against the register form.
# The ring form is not in the production library: build it first, e.g.
#   BCG_EXTRA_HIPFLAGS=-DPREFILL_LDS_BUILD=1 python -m byzantine_consensus_llm_agents_amd.utils.build --force
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
BCG_PREFILL_LDS=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py \
  -k "prefill" > gpurun_out/prefill_lds_tests.log 2>&1 || { tail -40 gpurun_out/prefill_lds_tests.log; exit 1; }
tail -2 gpurun_out/prefill_lds_tests.log
for r in 1 2; do
  for v in 0 1; do
    echo "== lds=$v"; BCG_PREFILL_LDS=$v timeout -k 10 120 python -u tools/bench_prefill.py --skip-gemm 2>&1 | grep attn || exit 1
  done
done
