#!/bin/bash
# silu_mul: GPU tests + bandwidth at prefill M (round 3).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "silu_mul" > gpurun_out/silu_tests.log 2>&1 || { tail -30 gpurun_out/silu_tests.log; exit 1; }
tail -2 gpurun_out/silu_tests.log
timeout -k 10 120 python - <<'PY'
import torch
from byzantine_consensus_llm_agents_amd.ops import get_ops
hip = get_ops("hip")
for T in (3000, 9000, 16384):
    gus = [torch.randn(T, 2 * 17408, device="cuda", dtype=torch.bfloat16) for _ in range(3)]
    for i in range(3): hip.silu_mul(gus[i])
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(30): hip.silu_mul(gus[i % 3])
    b.record(); b.synchronize()
    us = a.elapsed_time(b) / 30 * 1e3
    print(f"silu_mul T={T}: {us:.1f} us, {T * 17408 * 6 / us / 1e6:.2f} TB/s", flush=True)
PY
