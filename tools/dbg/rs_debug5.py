"""RS split-K debug: what the wrong j=7 values are made of (tools-only)."""
import ctypes
import os
import sys
import torch
sys.path.insert(0, ".")
from byzantine_consensus_llm_agents_amd.ops.hip import load_library, kernels_target
lib = load_library(os.environ.get("BCG_KERNELS_LIB") or kernels_target())
p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
cnt = torch.zeros(65536, dtype=torch.int32, device="cuda")
M, N, K = 256, 256, 4096
torch.manual_seed(0)
x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
ref = x.float() @ w.float().t()
nk = K // 64
for S in (6, 7, 8):
    parts = [x[:, s * nk // S * 64:(s + 1) * nk // S * 64].float() @ w[:, s * nk // S * 64:(s + 1) * nk // S * 64].float().t() for s in range(S)]
    for rep in range(2):
        ws = torch.full((S * 65536,), float("nan"), device="cuda")
        out = torch.zeros(M, N, dtype=torch.float32, device="cuda").to(torch.bfloat16)
        lib.bcg_gemm_w4(0, p(x), p(w), None, None, p(out), p(ws), p(cnt), M, N, K, N // 2, S, None)
        torch.cuda.synchronize()
        d = out.float() - ref
        bad = d.abs() > 0.1
        idx = bad.nonzero()
        if len(idx) == 0:
            print("S", S, "rep", rep, "clean"); continue
        rows = sorted(set(idx[:, 0].tolist())); cols = sorted(set(idx[:, 1].tolist()))
        print("S", S, "rep", rep, "bad", len(idx), "rows", rows[0], "..", rows[-1], len(rows), "cols", cols)
        # explain d by a signed subset of parts
        best = []
        for k in range(S):
            for sg in (1, -1):
                best.append(((d[bad] - sg * parts[k][bad]).abs().max().item(), "%+d*part%d" % (sg, k)))
        best.sort()
        print("   best single explanation", best[:3], " |d| max", d[bad].abs().max().item())
