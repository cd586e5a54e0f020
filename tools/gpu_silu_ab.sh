#!/bin/bash
# silu_mul A/B: build/libbcg_silu_old.so (1 row per thread-iteration) vs the in-tree library.
set -o pipefail
mkdir -p gpurun_out
cat > /tmp/silu_time.py <<'PY'
import os, torch
from byzantine_consensus_llm_agents_amd.ops import get_ops
hip = get_ops("hip")
tag = "old" if os.environ.get("BCG_KERNELS_LIB") else "new"
for T in (3000, 9000, 16384):
    gus = [torch.randn(T, 2 * 17408, device="cuda", dtype=torch.bfloat16) for _ in range(3)]
    for i in range(3): hip.silu_mul(gus[i])
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(30): hip.silu_mul(gus[i % 3])
    b.record(); b.synchronize()
    us = a.elapsed_time(b) / 30 * 1e3
    print(f"{tag} silu_mul T={T}: {us:.1f} us, {T * 17408 * 6 / us / 1e6:.2f} TB/s", flush=True)
PY
for r in 1 2; do
  BCG_KERNELS_LIB=$PWD/build/libbcg_silu_old.so PYTHONPATH=$PWD timeout -k 10 120 python /tmp/silu_time.py || exit 1
  PYTHONPATH=$PWD timeout -k 10 120 python /tmp/silu_time.py || exit 1
done
