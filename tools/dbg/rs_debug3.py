"""RS split-K debug: NaN-filled workspace (read-but-unwritten pieces show as NaN), slab check (tools-only)."""
import ctypes
import os
import sys
import torch
sys.path.insert(0, ".")
from byzantine_consensus_llm_agents_amd.ops.hip import load_library
lib = load_library(os.environ.get("BCG_KERNELS_LIB", "build/libbcg_rsd1.so"))
p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
M, N, K = 256, 256, 4096
torch.manual_seed(0)
x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
ref = x.float() @ w.float().t()
cnt = torch.zeros(65536, dtype=torch.int32, device="cuda")
for S in (2, 3, 4):
    ws = torch.full((S * 65536,), float("nan"), device="cuda")
    out = torch.zeros(M, N, dtype=torch.bfloat16, device="cuda")
    rc = lib.bcg_gemm_w4(0, p(x), p(w), None, None, p(out), p(ws), p(cnt), M, N, K, N // 2, S, None)
    torch.cuda.synchronize()
    e = (out.float() - ref).abs()
    nanrows = sorted(set(torch.isnan(out.float()).nonzero()[:, 0].tolist()))
    badrows = sorted(set((e > 0.1).nonzero()[:, 0].tolist()))
    print("S", S, "rc", rc, "max err", e.nan_to_num(99).max().item(), "nan rows", nanrows[:20], "bad rows", badrows[:40])
    # slab check: piece (sp, wave, i, j) = lane-major 256 floats of block (i = n-block, j = m-block)
    nk = K // 64
    slab = ws.view(S, 4, 8, 8, 64, 4)
    for sp in range(S):
        k0, k1 = sp * nk // S * 64, (sp + 1) * nk // S * 64
        part = x[:, k0:k1].float() @ w[:, k0:k1].float().t()
        jlo, jhi = sp * 8 // S, (sp + 1) * 8 // S
        worst = 0.0
        for wv in range(4):
            wm, wn = wv & 1, wv >> 1
            blk = part[wm * 128:(wm + 1) * 128, wn * 128:(wn + 1) * 128]  # [m, n]
            # lane l: fr = l & 15 (m row), fq = l >> 4 ; element e: n = 16 i + 4 fq + e ; m = 16 j + fr
            exp = blk.view(8, 16, 8, 4, 4).permute(2, 0, 3, 1, 4).reshape(8, 8, 64, 4)  # [i][j][lane][e]
            got = slab[sp, wv]
            for j in range(8):
                if jlo <= j < jhi:
                    continue
                worst = max(worst, (got[:, j] - exp[:, j]).abs().nan_to_num(99).max().item())
        print("   slab sp", sp, "stored pieces max err", worst)

print("---- detail")
for S in (2, 4):
    nk = K // 64
    parts = [x[:, sp * nk // S * 64:(sp + 1) * nk // S * 64].float() @ w[:, sp * nk // S * 64:(sp + 1) * nk // S * 64].float().t()
             for sp in range(S)]
    ws = torch.full((S * 65536,), float("nan"), device="cuda")
    out = torch.zeros(M, N, dtype=torch.bfloat16, device="cuda")
    lib.bcg_gemm_w4(0, p(x), p(w), None, None, p(out), p(ws), p(cnt), M, N, K, N // 2, S, None)
    torch.cuda.synchronize()
    d = out.float() - ref
    bad = d.abs() > 0.1
    idx = bad.nonzero()
    print("S", S, "bad count", int(bad.sum()), "rows", sorted(set(idx[:, 0].tolist()))[:3], "cols", sorted(set(idx[:, 1].tolist())))
    for sp in range(S):
        print("   d + part%d max" % sp, (d[bad] + parts[sp][bad]).abs().max().item(),
              " d - part%d max" % sp, (d[bad] - parts[sp][bad]).abs().max().item())
    slab = ws.view(S, 4, 8, 8, 64, 4)
    for sp in range(S):
        jlo, jhi = sp * 8 // S, (sp + 1) * 8 // S
        for wv in range(4):
            wm, wn = wv & 1, wv >> 1
            blk = parts[sp][wm * 128:(wm + 1) * 128, wn * 128:(wn + 1) * 128]
            exp = blk.view(8, 16, 8, 4, 4).permute(2, 0, 3, 1, 4).reshape(8, 8, 64, 4)
            for i in range(8):
                for j in range(8):
                    if jlo <= j < jhi:
                        continue
                    err = (slab[sp, wv, i, j] - exp[i, j]).abs().nan_to_num(99)
                    if err.max() > 0.01:
                        lanes = sorted(set((err > 0.01).nonzero()[:, 0].tolist()))
                        alt = [(o, (slab[sp, wv, i, j] - parts[o][wm * 128:(wm + 1) * 128, wn * 128:(wn + 1) * 128].view(8, 16, 8, 4, 4).permute(2, 0, 3, 1, 4).reshape(8, 8, 64, 4)[i, j]).abs().max().item()) for o in range(S)]
                        print("   bad slab piece sp", sp, "wave", wv, "i", i, "j", j, "lanes", lanes[:8], "...", len(lanes), "vs parts", alt,
                              "zero?", slab[sp, wv, i, j][err > 0.01][:4].tolist())
