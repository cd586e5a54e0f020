"""Micro-benchmarks of the decode hot ops on one MI355X (interleaved A/B in one process).

  python tools/bench_ops.py [--model qwen3-14b] [--ms 16,40,80,128,160,192]

Reports per-op time and effective HBM bandwidth (weight / KV bytes moved) for:
  * decode projections: the GEMM plan (hand kernel / library) vs torch.nn.functional.linear (hipBLASLt);
  * paged decode attention (bytes = K+V of every context token);
  * the fused guided sampler.
Writes a JSON summary to gpurun_out/bench_ops.json.
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


def timeit(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    start.record()
    for _ in range(iters):
        fn()
    end.record()
    torch.cuda.synchronize()
    return start.elapsed_time(end) / iters * 1e3  # us


def main():
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen3-14b")
    ap.add_argument("--ms", default="16,40,80,128,160,192")
    ap.add_argument("--ctx", type=int, default=1700)
    ap.add_argument("--tunable", action="store_true", help="PyTorch TunableOp for the hipBLASLt GEMMs")
    ap.add_argument("--skip-gemm", action="store_true")
    ap.add_argument("--share", type=int, default=1,
                    help="decode attention: rows in groups of this many map the same first 16 KV blocks "
                         "(the prefix cache's shared system-prompt blocks)")
    args = ap.parse_args()
    if args.tunable:
        torch.cuda.tunable.enable(True)
        torch.cuda.tunable.tuning_enable(True)
        torch.cuda.tunable.set_filename(os.path.join(ROOT, "gpurun_out", "tunableop_results.csv"))
    hip = get_ops("hip")
    cfg = get_model_config(args.model)
    H, I, hd = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
    shapes = {"qkv": ((cfg.num_heads + 2 * cfg.num_kv_heads) * hd, H), "o": (H, cfg.num_heads * hd),
              "gate_up": (2 * I, H), "down": (H, I), "lm_head": (cfg.vocab_size, H)}
    weights = {k: torch.randn(n, kk, device="cuda", dtype=torch.bfloat16) * 0.02 for k, (n, kk) in shapes.items()}
    out = {"model": cfg.name, "gemm": [], "attention": [], "sample": []}
    for M in ([] if args.skip_gemm else [int(m) for m in args.ms.split(",")]):
        x = {k: torch.randn(M, kk, device="cuda", dtype=torch.bfloat16) for k, (n, kk) in shapes.items()}
        for name, w in weights.items():
            t_pl = timeit(lambda: hip.linear(x[name], w))
            t_bl = timeit(lambda: torch.nn.functional.linear(x[name], w))
            gb = w.numel() * 2 / 1e9
            rec = {"M": M, "op": name, "plan_us": round(t_pl, 1), "hipblaslt_us": round(t_bl, 1),
                   "plan_TBps": round(gb / t_pl * 1e3, 2), "hipblaslt_TBps": round(gb / t_bl * 1e3, 2)}
            out["gemm"].append(rec)
            print(json.dumps(rec), flush=True)
    # decode attention at the bench geometry
    b_list = [int(b) for b in os.environ.get("BCG_BENCH_B", "8,40,160,192").split(",")]
    NB = 1 + (args.ctx // 16 + 1) * max(b_list)  # every row's table must stay inside the cache
    k = torch.randn(1, NB, cfg.num_kv_heads, 16, hd, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(1, NB, cfg.num_kv_heads, hd, 16, device="cuda", dtype=torch.bfloat16)
    for B in b_list:
        nb = (args.ctx + 15) // 16
        assert B * nb + 1 <= NB
        tables = (torch.arange(B * nb, dtype=torch.int32, device="cuda").view(B, nb) + 1)
        if args.share > 1:  # every row of a group maps the group leader's first 16 blocks
            lead = (torch.arange(B, device="cuda") // args.share) * args.share
            tables[:, :16] = tables[lead, :16]
        tables = torch.cat([tables, torch.zeros(B, 512 - nb, dtype=torch.int32, device="cuda")], 1).contiguous()
        seq = torch.full((B,), args.ctx, dtype=torch.int32, device="cuda")
        q = torch.randn(B, cfg.num_heads, hd, device="cuda", dtype=torch.bfloat16)
        t = timeit(lambda: hip.paged_attention_decode(q, k, v, 0, tables, seq, hd ** -0.5))
        gb = B * args.ctx * cfg.num_kv_heads * hd * 2 * 2 / 1e9
        rec = {"B": B, "ctx": args.ctx, "share": args.share, "us": round(t, 1), "TBps": round(gb / t * 1e3, 2)}
        out["attention"].append(rec)
        print(json.dumps(rec), flush=True)
    # fused QK-norm + RoPE + paged KV write (decode rows and a prefill chunk)
    from byzantine_consensus_llm_agents_amd.ops.reference import rope_cache
    cs = rope_cache(8192, hd, 1e6, "cuda")
    n_q, n_kv = cfg.num_heads, cfg.num_kv_heads
    out["rope"] = []
    for T, in_order in ((616, False), (16384, False), (16384, True)):  # in order: a prefill chunk's blocks
        nbk = T // 16 + 2
        kc = torch.zeros(1, nbk, n_kv, 16, hd, device="cuda", dtype=torch.bfloat16)
        vc = torch.zeros(1, nbk, n_kv, hd, 16, device="cuda", dtype=torch.bfloat16)
        qkv = torch.randn(T, (n_q + 2 * n_kv) * hd, device="cuda", dtype=torch.bfloat16)
        pos = torch.randint(0, 4000, (T,), device="cuda", dtype=torch.int32)
        slots = (torch.arange(16, 16 + T, device="cuda") if in_order
                 else torch.randperm(nbk * 16, device="cuda")[:T]).to(torch.int32)
        wn = torch.ones(hd, device="cuda", dtype=torch.bfloat16)
        t = timeit(lambda: hip.qk_norm_rope_kv_write(qkv, pos, slots, n_q, n_kv, hd, wn, wn, 1e-6, cs, kc, vc, 0))
        gb = (qkv.numel() * 2 + T * n_q * hd * 2 + T * 2 * n_kv * hd * 2) / 1e9
        rec = {"T": T, "in_order": in_order, "rope_us": round(t, 1), "TBps": round(gb / t * 1e3, 2)}
        out["rope"].append(rec)
        print(json.dumps(rec), flush=True)
    # sampler
    V = cfg.vocab_size
    for B in (40, 160):
        logits = torch.randn(B, V, device="cuda", dtype=torch.bfloat16)
        nxt = torch.randint(-1, 100, (128, V), device="cuda", dtype=torch.int16)
        dist = torch.randint(0, 50, (128,), device="cuda", dtype=torch.int16)
        st = {n: torch.zeros(B, dtype=torch.int32, device="cuda") for n in
              ("fsm_base", "fsm_state", "gen_count", "row_keys", "done", "seq_lens", "next_tokens")}
        mx = torch.full((B,), 1 << 30, dtype=torch.int32, device="cuda")
        temp = torch.full((B,), 0.5, device="cuda")
        outt = torch.zeros(B, 1 << 14, dtype=torch.int32, device="cuda")

        def run():
            st["gen_count"].zero_()
            hip.sample_step(logits, nxt, dist, st["fsm_base"], st["fsm_state"], st["gen_count"], mx, temp,
                            st["row_keys"], st["done"], st["seq_lens"], outt, st["next_tokens"], 7, True,
                            V - 500, 0, 1)
        t = timeit(run)
        rec = {"B": B, "V": V, "us": round(t, 1)}
        out["sample"].append(rec)
        print(json.dumps(rec), flush=True)
    if args.tunable:
        torch.cuda.tunable.write_file() if hasattr(torch.cuda.tunable, "write_file") else None
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "bench_ops.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
