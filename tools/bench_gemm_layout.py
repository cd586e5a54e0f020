"""Projection GEMM rate vs weight layout on one MI355X (hipBLASLt and rocBLAS).

  python tools/bench_gemm_layout.py [--model qwen3-14b] [--m 16384,8192,448]

y = x W^T with W stored [N, K] (torch Linear layout: hipBLASLt "TN") versus W
stored transposed [K, N] contiguous ("NN": y = x @ Wt).  Prints TF/s per shape
and layout and writes gpurun_out/bench_gemm_layout.json.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from byzantine_consensus_llm_agents_amd.models.config import get_model_config  # noqa: E402


def timeit(fn, iters=10, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen3-14b")
    ap.add_argument("--m", default="16384,8192,448")
    args = ap.parse_args()
    cfg = get_model_config(args.model)
    H, I, hd = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
    shapes = {"qkv": ((cfg.num_heads + 2 * cfg.num_kv_heads) * hd, H), "o": (H, cfg.num_heads * hd),
              "gate_up": (2 * I, H), "down": (H, I)}
    out = []
    for lib in ("cublaslt", "cublas"):
        torch.backends.cuda.preferred_blas_library(lib)
        for M in [int(m) for m in args.m.split(",")]:
            for name, (N, K) in shapes.items():
                w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
                wt = w.t().contiguous()
                x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
                for layout, fn in (("tn", lambda: torch.nn.functional.linear(x, w)),
                                   ("nn", lambda: torch.matmul(x, wt))):
                    us = timeit(fn)
                    tf = 2 * M * N * K / us / 1e6
                    out.append({"lib": lib, "M": M, "op": name, "N": N, "K": K, "layout": layout,
                                "us": round(us, 1), "tflops": round(tf, 1)})
                    print(f"[{lib:8s}] M={M:6d} {name:8s} {layout} {us:9.1f} us {tf:7.1f} TF/s", flush=True)
                del w, wt, x
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "bench_gemm_layout.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
