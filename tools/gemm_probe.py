"""One hand-GEMM (or library) configuration in a loop, for rocprofv3 PMC passes.

  python tools/gemm_probe.py --m 768 --n 34816 --k 5120 --epi 1 --cfg 8 --split 1 [--lib] [--iters 50]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from byzantine_consensus_llm_agents_amd.ops import get_ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=768)
    ap.add_argument("--n", type=int, default=34816)
    ap.add_argument("--k", type=int, default=5120)
    ap.add_argument("--epi", type=int, default=1)
    ap.add_argument("--cfg", type=int, default=8)
    ap.add_argument("--split", type=int, default=1)
    ap.add_argument("--lib", action="store_true")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    hip = get_ops("hip")
    ws = [torch.randn(a.n, a.k, device="cuda").mul_(a.k ** -0.5).to(torch.bfloat16) for _ in range(3)]
    x = torch.randn(a.m, a.k, device="cuda").to(torch.bfloat16)
    r = torch.randn(a.m, a.n, device="cuda").to(torch.bfloat16)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for it in range(a.iters + 5):
        if it == 5:
            ev[0].record()
        w = ws[it % 3]
        if a.lib:
            F.linear(x, w)
        elif a.epi == 2:
            hip.gemm_nt(x, w, a.cfg, 2, residual=r, out=r, split_k=a.split)
        else:
            hip.gemm_nt(x, w, a.cfg, a.epi, split_k=a.split)
    ev[1].record()
    ev[1].synchronize()
    us = ev[0].elapsed_time(ev[1]) * 1e3 / a.iters
    print(f"{'lib' if a.lib else f'cfg{a.cfg}x{a.split}'} M={a.m} N={a.n} K={a.k}: {us:.1f} us "
          f"{2 * a.m * a.n * a.k / us / 1e6:.0f} TF/s")


if __name__ == "__main__":
    main()
