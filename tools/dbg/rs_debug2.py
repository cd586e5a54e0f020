"""RS split-K debug: which split's partial is missing in the bad block (tools-only)."""
import sys
import torch
sys.path.insert(0, ".")
from byzantine_consensus_llm_agents_amd.ops import get_ops
hip = get_ops("hip")
M, N, K = 256, 1024, 4096
torch.manual_seed(0)
x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
ref = x.float() @ w.float().t()
for S in (3, 4):
    nk = K // 64
    parts = []
    for s in range(S):
        k0, k1 = s * nk // S * 64, (s + 1) * nk // S * 64
        parts.append(x[:, k0:k1].float() @ w[:, k0:k1].float().t())
    got = hip.gemm_nt(x, w, 11, 0, split_k=S).float()
    d = got - ref
    bad = d.abs() > 0.1
    print("S", S, "bad", int(bad.sum()), "rows", sorted(set(bad.nonzero()[:, 0].tolist()))[:40])
    print("  cols", sorted(set(bad.nonzero()[:, 1].tolist()))[:64])
    for s in range(S):
        r = (d[bad] + parts[s][bad]).abs().max().item() if bad.any() else 0
        r2 = (d[bad] - parts[s][bad]).abs().max().item() if bad.any() else 0
        print("  |d + part%d| max %.3f   |d - part%d| max %.3f" % (s, r, s, r2))
    print("  d sample", d[bad][:8].tolist())
    print("  got sample", got[bad][:8].tolist())
