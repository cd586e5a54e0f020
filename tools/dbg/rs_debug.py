"""RS split-K debug: error per 16-row m-block for splits 2..8 (tools-only)."""
import sys
import torch
sys.path.insert(0, ".")
from byzantine_consensus_llm_agents_amd.ops import get_ops
hip = get_ops("hip")
for M, N, K in [(150, 1024, 4096), (256, 1024, 4096), (704, 1024, 5120)]:
    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    ref = x.float() @ w.float().t()
    for sp in range(2, 9):
        got = hip.gemm_nt(x, w, 11, 0, split_k=sp).float()
        e = (got - ref).abs()
        rows = e.max(dim=1).values
        blk = [round(rows[i:i + 16].max().item(), 2) for i in range(0, min(M, 256), 16)]
        cols = e.max(dim=0).values
        print(M, N, K, "split", sp, "max", round(e.max().item(), 3), "rowblocks", blk,
              "bad cols", int((cols > 0.1).sum()), flush=True)
