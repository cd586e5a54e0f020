"""Decode attention with and without the shared-prefix cascade (one MI355X, interleaved A/B).

  python tools/bench_cascade.py [--model qwen3-14b] [--b 256,608] [--shared 40] [--own 1100] [--group 24]

Rows come in groups of `--group` that map the same `--shared` leading KV blocks (the
prefix cache's system-prompt blocks: ~40 blocks = 648 tokens per row in the driver's
bench) followed by `--own` private tokens.  Times per layer: the per-row kernel alone
(reads every row's shared blocks; L2 / MALL may catch repeats), and the cascade (shared
blocks once per group + own tokens per row).  Writes gpurun_out/bench_cascade.json.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from byzantine_consensus_llm_agents_amd.engine.cascade import CascadeTables, plan_groups  # noqa: E402
from byzantine_consensus_llm_agents_amd.models.config import get_model_config  # noqa: E402
from byzantine_consensus_llm_agents_amd.ops import get_ops  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen3-14b")
    ap.add_argument("--b", default="256,608")
    ap.add_argument("--shared", default="20,40")
    ap.add_argument("--own", type=int, default=1100)
    ap.add_argument("--group", default="8,24,64")
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    hip = get_ops("hip")
    cfg = get_model_config(args.model)
    n_q, n_kv, hd = cfg.num_heads, cfg.num_kv_heads, cfg.head_dim
    bs = [int(x) for x in args.b.split(",")]
    shareds = [int(x) for x in args.shared.split(",")]
    gsizes = [int(x) for x in args.group.split(",")]
    own_blk = (args.own + 200 + 15) // 16  # own tokens vary by +-200
    max_blocks = max(shareds) + own_blk + 1
    NB = 2 + max(bs) * (max(shareds) + own_blk + 1)
    k = torch.randn(1, NB, n_kv, 16, hd, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(1, NB, n_kv, hd, 16, device="cuda", dtype=torch.bfloat16)
    gen = torch.Generator().manual_seed(0)
    res = []
    for B in bs:
        ws = torch.empty(hip.decode_workspace_numel(B, n_q, hd, max_blocks), dtype=torch.float32, device="cuda")
        q = torch.randn(B, n_q, hd, device="cuda", dtype=torch.bfloat16)
        for S in shareds:
            for gsz in gsizes:
                nxt = 1
                rows, lens = [], []
                for r in range(B):
                    if r % gsz == 0:
                        common = list(range(nxt, nxt + S))
                        nxt += S
                    own = args.own + int(torch.randint(-200, 200, (1,), generator=gen))
                    nb = (own + 15) // 16
                    rows.append(common + list(range(nxt, nxt + nb)))
                    nxt += nb
                    lens.append(S * 16 + own)
                assert nxt <= NB
                perm = torch.randperm(B, generator=gen).tolist()  # groups interleaved over rows
                rows, lens = [rows[i] for i in perm], [lens[i] for i in perm]
                tables = torch.zeros(B, max_blocks, dtype=torch.int32)
                for r, blks in enumerate(rows):
                    tables[r, :len(blks)] = torch.tensor(blks, dtype=torch.int32)
                tables = tables.cuda()
                seq = torch.tensor(lens, dtype=torch.int32, device="cuda")
                cas = CascadeTables(B, "cuda")
                cas.upload(plan_groups(list(enumerate(rows))), n_q // n_kv)
                t_plain, t_cas = [], []
                for _ in range(args.rounds):
                    t_plain.append(timeit(lambda: hip.paged_attention_decode(q, k, v, 0, tables, seq, hd ** -0.5, ws)))
                    t_cas.append(timeit(lambda: hip.paged_attention_decode(q, k, v, 0, tables, seq, hd ** -0.5, ws,
                                                                           cas)))
                a = hip.paged_attention_decode(q, k, v, 0, tables, seq, hd ** -0.5, ws)
                b = hip.paged_attention_decode(q, k, v, 0, tables, seq, hd ** -0.5, ws, cas)
                err = (a.float() - b.float()).abs().max().item()
                kv_gb = sum(lens) * n_kv * hd * 4 / 1e9   # K + V bytes of every row's context
                rec = {"B": B, "shared_blocks": S, "group": gsz, "mean_ctx": round(sum(lens) / B),
                       "plain_us": round(min(t_plain), 1), "cascade_us": round(min(t_cas), 1),
                       "speedup": round(min(t_plain) / min(t_cas), 3),
                       "plain_TBps_logical": round(kv_gb / min(t_plain) * 1e3, 2),
                       "cascade_TBps_logical": round(kv_gb / min(t_cas) * 1e3, 2),
                       "groups": len(cas.groups), "items": int(cas.n_items[0]), "max_abs_diff": err}
                res.append(rec)
                print(json.dumps(rec), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "bench_cascade.json"), "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
