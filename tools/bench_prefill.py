"""Prefill-shaped op micro-benchmarks on one MI355X (TFLOP/s per GEMM shape, attention).

  python tools/bench_prefill.py [--model qwen3-14b] [--m 16384]

GEMMs: y = x W^T for every projection of the model at M prefill tokens, timed
with (a) hipBLASLt default heuristics, (b) the engine's shipped TunableOp
table, (c) rocBLAS (torch's "cublas" preference on ROCm).  Attention: the HIP
paged prefill kernel on packed prompts of `--prompt` tokens each with a
cached prefix of `--prefix` tokens.  JSON -> gpurun_out/bench_prefill.json.
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


def gemms(cfg, M, mode):
    H, I, hd = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
    shapes = {"qkv": ((cfg.num_heads + 2 * cfg.num_kv_heads) * hd, H), "o": (H, cfg.num_heads * hd),
              "gate_up": (2 * I, H), "down": (H, I)}
    res = {}
    for name, (N, K) in shapes.items():
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        us = timeit(lambda: torch.nn.functional.linear(x, w))
        res[name] = {"N": N, "K": K, "us": round(us, 1), "tflops": round(2 * M * N * K / us / 1e6, 1)}
        print(f"[{mode}] M={M} {name:8s} N={N:6d} K={K:6d} {us:9.1f} us {res[name]['tflops']:7.1f} TF/s",
              flush=True)
    tot_us = sum(r["us"] for r in res.values())
    flops = sum(2 * M * r["N"] * r["K"] for r in res.values())
    print(f"[{mode}] layer total {tot_us:.0f} us = {flops / tot_us / 1e6:.0f} TF/s", flush=True)
    return res


def attention(cfg, n_prompts, prompt, prefix, tile_rows=64):
    from byzantine_consensus_llm_agents_amd.ops import get_ops
    hip = get_ops("hip")
    bs, hd = 16, cfg.head_dim
    n_q, n_kv = cfg.num_heads, cfg.num_kv_heads
    ctx = prefix + prompt
    nb_seq = (ctx + bs - 1) // bs
    NB = n_prompts * nb_seq + 1
    k = torch.randn(1, NB, n_kv, bs, hd, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(1, NB, n_kv, hd, bs, device="cuda", dtype=torch.bfloat16)
    tables = (torch.arange(n_prompts * nb_seq, dtype=torch.int32) + 1).view(n_prompts, nb_seq).cuda()
    q_start = torch.arange(n_prompts + 1, dtype=torch.int32) * prompt
    tiles = []
    for i in range(n_prompts):
        for t in range(i * prompt, (i + 1) * prompt, tile_rows):
            tiles.append((i, t, min(t + tile_rows, (i + 1) * prompt)))
    tiles.sort(key=lambda x: -(x[2] - x[0] * prompt))  # deepest first, as the engine orders them
    tiles = torch.tensor(tiles, dtype=torch.int32).cuda()
    T = n_prompts * prompt
    q = torch.randn(T, n_q, hd, device="cuda", dtype=torch.bfloat16)
    seq_lens = torch.full((n_prompts,), ctx, dtype=torch.int32, device="cuda")
    us = timeit(lambda: hip.paged_attention_prefill(q, k, v, 0, tables, q_start.cuda(), seq_lens, hd ** -0.5,
                                                    prompt, tiles, tile_rows=tile_rows))
    # causal FLOPs: each query sees prefix + its causal part
    flops = 4 * n_q * hd * n_prompts * (prompt * prefix + prompt * (prompt + 1) / 2)
    r = {"prompts": n_prompts, "prompt": prompt, "prefix": prefix, "tile_rows": tile_rows, "us": round(us, 1),
         "tflops": round(flops / us / 1e6, 1)}
    print(f"[attn rows={tile_rows}] {n_prompts}x{prompt} (+{prefix} cached) {us:9.1f} us {r['tflops']:7.1f} TF/s",
          flush=True)
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen3-14b")
    ap.add_argument("--m", default="16384")
    ap.add_argument("--modes", default="default,tuned,rocblas")
    ap.add_argument("--skip-gemm", action="store_true")
    ap.add_argument("--skip-attn", action="store_true")
    ap.add_argument("--attn-model", default=None, help="model geometry for the attention runs")
    ap.add_argument("--tile-rows", default="64", help="prefill attention tile sizes to time (64,128,256)")
    ap.add_argument("--attn-shapes", default="12x1024+512,16x900+400,8x2048+0",
                    help="prompts x new tokens + cached prefix")
    args = ap.parse_args()
    cfg = get_model_config(args.model)
    out = {"model": cfg.name, "gemm": {}, "attention": []}
    for mode in ([] if args.skip_gemm else args.modes.split(",")):
        if mode == "tuned":
            name = cfg.name.split("/")[-1].lower()
            path = os.path.join(ROOT, "byzantine_consensus_llm_agents_amd", "engine", "tuned",
                                f"tunableop_{name}_tp1.csv")
            t = torch.cuda.tunable
            t.enable(True)
            t.tuning_enable(False)
            t.set_filename(os.path.join("/tmp", f"bench_prefill_tunable_{os.getpid()}.csv"))
            t.read_file(path)
        elif mode == "rocblas":
            torch.cuda.tunable.enable(False)
            torch.backends.cuda.preferred_blas_library("cublas")
        for M in [int(m) for m in args.m.split(",")]:
            out["gemm"][f"{mode}_M{M}"] = gemms(cfg, M, mode)
        torch.backends.cuda.preferred_blas_library("cublaslt")
        torch.cuda.tunable.enable(False)
    acfg = get_model_config(args.attn_model) if args.attn_model else cfg
    shapes = []
    for spec in args.attn_shapes.split(","):
        n, rest = spec.split("x")
        p, pre = rest.split("+")
        shapes.append((int(n), int(p), int(pre)))
    for n, p, pre in (() if args.skip_attn else shapes):
        for tr in (int(x) for x in args.tile_rows.split(",")):
            out["attention"].append(attention(acfg, n, p, pre, tr))
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "bench_prefill.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
