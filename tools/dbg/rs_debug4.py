"""RS split-K debug: NaN workspace, 4 tiles, splits 2..8 in sequence (tools-only)."""
import ctypes
import os
import sys
import torch
sys.path.insert(0, ".")
from byzantine_consensus_llm_agents_amd.ops.hip import load_library, kernels_target
lib = load_library(os.environ.get("BCG_KERNELS_LIB") or kernels_target())
p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
cnt = torch.zeros(65536, dtype=torch.int32, device="cuda")
for M, N, K in [(150, 1024, 4096), (256, 1024, 4096)]:
    torch.manual_seed(0)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    ref = x.float() @ w.float().t()
    tiles = (M + 255) // 256 * (N // 256)
    for S in range(2, 9):
        ws = torch.full((tiles * S * 65536,), float("nan"), device="cuda")
        out = torch.zeros(M, N, dtype=torch.bfloat16, device="cuda")
        rc = lib.bcg_gemm_w4(0, p(x), p(w), None, None, p(out), p(ws), p(cnt), M, N, K, N // 2, S, None)
        torch.cuda.synchronize()
        e = (out.float() - ref).abs()
        nanpos = torch.isnan(out.float()).nonzero()
        bad = (e.nan_to_num(99) > 0.1).nonzero()
        print(M, N, K, "S", S, "rc", rc, "nan", len(nanpos), "bad", len(bad),
              "tiles(n) with bad", sorted(set((bad[:, 1] // 256).tolist())), "rows", sorted(set(bad[:, 0].tolist()))[:4],
              "gen/cnt", cnt[65024:65024 + 2 * tiles].tolist(), flush=True)
