"""A/B of the prefill projection GEMMs: register-fed W4R (gemm_w4r.hip) vs LDS-fed W4 (gemm_w4.hip,
GEMM config 11) vs hipBLASLt, with the same epilogue work, interleaved in one process.

  python tools/bench_w4r.py [--model qwen3-14b] [--m 4096,8192,16384] [--reps 15]

qkv: y = x W^T; gate_up: silu(x Wg^T) * (x Wu^T); o / down: r += x W^T.  Weights rotate over
copies that exceed the 256 MiB Infinity Cache; median of --reps CUDA-event-timed calls per
candidate, candidates interleaved per repetition.  One JSON line per (projection, M).
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from byzantine_consensus_llm_agents_amd.models.config import get_model_config  # noqa: E402
from byzantine_consensus_llm_agents_amd.ops import get_ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen3-14b")
    ap.add_argument("--m", default="4096,8192,16384")
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--skip", default="")
    args = ap.parse_args()
    os.environ["BCG_HAND_GEMM"] = "0"
    hip = get_ops("hip")
    cfg = get_model_config(args.model)
    H, hd, I = cfg.hidden_size, cfg.head_dim, cfg.intermediate_size
    shapes = {"qkv": ((cfg.num_heads + 2 * cfg.num_kv_heads) * hd, H, 0), "o": (H, cfg.num_heads * hd, 2),
              "gate_up": (2 * I, H, 1), "down": (H, I, 2)}
    gen = torch.Generator(device="cuda").manual_seed(0)
    for proj, (N, K, epi) in shapes.items():
        if proj in args.skip.split(","):
            continue
        copies = max(2, min(6, -(-(1 << 30) // (N * K * 2))))
        ws = [torch.randn(N, K, device="cuda", generator=gen).mul_(K ** -0.5).to(torch.bfloat16) for _ in range(copies)]
        wr = [hip.w4r_weight(w, silu=epi == 1) for w in ws]
        for M in map(int, args.m.split(",")):
            x = torch.randn(M, K, device="cuda", generator=gen).to(torch.bfloat16)
            r = torch.randn(M, N, device="cuda", generator=gen).to(torch.bfloat16) if epi == 2 else None
            it = [0]

            def nxt():
                it[0] = (it[0] + 1) % copies
                return it[0]
            if epi == 0:
                fns = {"w4r": lambda: hip.gemm_w4r(x, wr[nxt()]), "w4": lambda: hip.gemm_nt(x, ws[nxt()], 11, 0),
                       "lib": lambda: F.linear(x, ws[nxt()])}
            elif epi == 1:
                fns = {"w4r": lambda: hip.gemm_w4r(x, wr[nxt()], epi=1), "w4": lambda: hip.gemm_nt(x, ws[nxt()], 11, 1),
                       "lib": lambda: hip.silu_mul(F.linear(x, ws[nxt()]))}
            else:
                fns = {"w4r": lambda: hip.gemm_w4r(x, wr[nxt()], epi=2, residual=r, out=r),
                       "w4": lambda: hip.gemm_nt(x, ws[nxt()], 11, 2, residual=r, out=r),
                       "lib": lambda: r.addmm_(x, ws[nxt()].t())}
            # correctness: W4R against W4 (same accumulation order: bitwise) on copy 0
            if epi == 2:
                a = hip.gemm_w4r(x, wr[0], epi=2, residual=r.clone(), out=torch.empty_like(r))
                b = hip.gemm_nt(x, ws[0], 11, 2, residual=r.clone(), out=torch.empty_like(r))
            else:
                a, b = hip.gemm_w4r(x, wr[0], epi=epi), hip.gemm_nt(x, ws[0], 11, epi)
            same = bool(torch.equal(a, b))
            for fn in fns.values():
                for _ in range(3):
                    fn()
            torch.cuda.synchronize()
            t = {k: [] for k in fns}
            for _ in range(args.reps):
                for k, fn in fns.items():
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    fn()
                    e1.record()
                    e1.synchronize()
                    t[k].append(e0.elapsed_time(e1) * 1e3)
            med = {k: round(statistics.median(v), 1) for k, v in t.items()}
            fl = 2.0 * M * N * K
            print(json.dumps({"proj": proj, "M": M, "N": N, "K": K, "us": med, "bitwise_w4": same,
                              "pf_s": {k: round(fl / v / 1e9, 3) for k, v in med.items()}}), flush=True)
        del ws, wr
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
