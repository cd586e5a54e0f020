"""fp8 projection GEMMs: every hand fp8 tile x split-K vs hipBLASLt (_scaled_mm); at prefill M
(> 1024) only the 256x256 kernels (cfg 10 ping-pong, cfg 11 four-wave).

  python tools/bench_fp8_gemm.py [--model mistral-22b] [--ms 32,64,128,160,256,320,512]

Weights are rotated over enough copies to fall out of the Infinity Cache.  Prints one
line per (projection, M) and writes gpurun_out/bench_fp8_gemm.json.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from byzantine_consensus_llm_agents_amd.models.config import get_model_config  # noqa: E402
from byzantine_consensus_llm_agents_amd.ops import get_ops  # noqa: E402
from byzantine_consensus_llm_agents_amd.ops.reference import quant_fp8  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mistral-22b")
    ap.add_argument("--ms", default="32,64,128,160,256,320,512")
    ap.add_argument("--tp", type=int, default=1, help="tensor-parallel degree of the shard shapes")
    args = ap.parse_args()
    cfg = get_model_config(args.model)
    hip = get_ops("hip")
    H, I, tp = cfg.hidden_size, cfg.intermediate_size // args.tp, args.tp
    hd = cfg.head_dim or H // cfg.num_heads
    nq, nkv = cfg.num_heads // tp, cfg.num_kv_heads // tp
    shapes = {"qkv": ((nq + 2 * nkv) * hd, H), "o": (H, nq * hd), "gate_up": (2 * I, H), "down": (H, I)}
    out = {}
    for name, (N, K) in shapes.items():
        copies = max(2, int(1.2e9 // (N * K)))
        ws_ = [quant_fp8((torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)) for _ in range(copies)]
        for M in map(int, args.ms.split(",")):
            xq, xs = quant_fp8(torch.randn(M, K, device="cuda").to(torch.bfloat16))
            it = [0]

            def nxt():
                it[0] = (it[0] + 1) % copies
                return ws_[it[0]]

            def lib():
                wq, wsc = nxt()
                return torch._scaled_mm(xq, wq.t(), scale_a=xs.view(-1, 1), scale_b=wsc.view(1, -1),
                                        out_dtype=torch.bfloat16)
            res = {"lib": timed(lib)}
            for c in range(12):  # 10 / 11 = the 256 x 256 ping-pong / four-wave kernels (N % 16)
                bm, bn = hip.gemm_plan.tiles[c]
                if N % (16 if c >= 10 else bn) or (M > 1024 and c < 10):
                    continue
                for sk in (1, 2, 3, 4, 6):
                    if K // 128 < sk or (M > 1024 and sk > 1):
                        continue
                    def hand(c=c, sk=sk):
                        wq, wsc = nxt()
                        return hip.gemm_nt_fp8(xq, xs, wq, wsc, (c, sk))
                    res[f"{c}x{sk}"] = timed(hand)
            best = min((v, k) for k, v in res.items() if k != "lib")
            tf = 2 * M * N * K / best[0] / 1e6
            print(f"{name:8s} M={M:4d} N={N:6d} K={K:5d} lib={res['lib']:8.1f}us best={best[1]:>5s} {best[0]:8.1f}us "
                  f"({tf:6.0f} TF/s, x{res['lib'] / best[0]:4.2f})", flush=True)
            out[f"{M},{N},{K}"] = {k: round(v, 2) for k, v in res.items()}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"bench_fp8_gemm_tp{args.tp}.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
