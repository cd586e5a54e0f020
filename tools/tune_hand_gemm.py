"""Measure the hand MFMA GEMM against hipBLASLt on decode shapes; write the dispatch table.

  python tools/tune_hand_gemm.py --model qwen3-14b [--tp 1] [--m 64,128,256,448,768]
         [--out byzantine_consensus_llm_agents_amd/engine/tuned/hand_gemm.json] [--merge]

For every decode M and every projection of the model, times each hand-kernel
tile configuration and the library path with the SAME epilogue work:
  qkv / lm_head : y = x W^T                    (library: F.linear)
  gate_up       : h = silu(x Wg^T) * (x Wu^T)  (library: F.linear + silu_mul kernel)
  o / down      : r = r + x W^T                (library: F.linear + add)
The library path uses the shipped TunableOp table (what the engine runs).
Weights rotate over enough copies to exceed the 256 MiB Infinity Cache, so
every call streams its weights from HBM as in a real decode step.  Median of
--reps timed calls per candidate (CUDA events), after a correctness check.
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

from byzantine_consensus_llm_agents_amd.models.config import ALIASES, get_model_config  # noqa: E402
from byzantine_consensus_llm_agents_amd.ops import get_ops  # noqa: E402
from byzantine_consensus_llm_agents_amd.ops.gemm_plan import BIG_CFGS, N_CFGS, SPLITS, STREAM_K, TABLE, W4_CFG  # noqa: E402


def shapes(cfg, tp):
    H, hd = cfg.hidden_size, cfg.head_dim
    nq, nkv, inter = cfg.num_heads // tp, cfg.num_kv_heads // tp, cfg.intermediate_size // tp
    return {"qkv": ((nq + 2 * nkv) * hd, H, 0), "o": (H, nq * hd, 2), "gate_up": (2 * inter, H, 1),
            "down": (H, inter, 2), "lm_head": (cfg.vocab_size // tp, H, 0)}


def timed(fn, reps):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen3-14b")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--m", default="16,32,64,96,128,160,224,256,320,384,448,512,576,640,704,768")
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--out", default=None)
    ap.add_argument("--merge", action="store_true", help="add to the existing table instead of replacing it")
    ap.add_argument("--skip", default="", help="comma list of projections to skip")
    ap.add_argument("--cfgs", default="", help="comma list of tile configurations to time (default: all); "
                    "with --merge the table's previous best configuration is timed again as well")
    args = ap.parse_args()
    only_cfgs = {int(c) for c in args.cfgs.split(",") if c}
    os.environ["BCG_HAND_GEMM"] = "0"  # the library path of linear() must not dispatch to us
    hip = get_ops("hip")
    name = ALIASES.get(args.model, args.model).split("/")[-1].lower()
    tuned = os.path.join(ROOT, "byzantine_consensus_llm_agents_amd", "engine", "tuned",
                         f"tunableop_{name}_tp{args.tp}.csv")
    if os.path.exists(tuned):
        t = torch.cuda.tunable
        t.enable(True)
        t.tuning_enable(False)
        t.set_filename(f"/tmp/bcg_tune_hand_{os.getpid()}.csv")
        t.read_file(tuned)
    cfg = get_model_config(args.model)
    out_path = args.out or os.path.join(ROOT, "gpurun_out", "hand_gemm.json")
    table = {"choice": {}, "timings_us": {}}
    if args.merge and os.path.exists(TABLE):
        with open(TABLE) as fh:
            table = json.load(fh)
    Ms = [int(m) for m in args.m.split(",")]
    skip = set(filter(None, args.skip.split(",")))
    gen = torch.Generator(device="cuda").manual_seed(0)
    for proj, (N, K, epi) in shapes(cfg, args.tp).items():
        if proj in skip:
            continue
        wbytes = N * K * 2
        copies = max(2, -(-(1 << 30) // wbytes))
        ws = [torch.randn(N, K, device="cuda", generator=gen).mul_(K ** -0.5).to(torch.bfloat16)
              for _ in range(min(copies, 8))]
        for M in Ms:
            if M > 1024 and proj == "lm_head":  # prefill computes logits of the last tokens only
                continue
            x = torch.randn(M, K, device="cuda", generator=gen).to(torch.bfloat16)
            r = torch.randn(M, N, device="cuda", generator=gen).to(torch.bfloat16) if epi == 2 else None
            it = [0]

            def w_next():
                it[0] = (it[0] + 1) % len(ws)
                return ws[it[0]]

            if epi == 0:
                lib = lambda: F.linear(x, w_next())  # noqa: E731
            elif epi == 1:
                lib = lambda: hip.silu_mul(F.linear(x, w_next()))  # noqa: E731
            else:
                lib = lambda: r.addmm_(x, w_next().t())  # noqa: E731  (the engine's library path: beta = 1 epilogue)
            ref = F.linear(x, ws[0]).float()
            if epi == 1:
                ref = F.silu(ref[:, :N // 2]) * ref[:, N // 2:]
            res = {"lib": None}
            for _ in range(3):
                lib()
            res["lib"] = timed(lib, args.reps)
            key = f"{M},{N},{K},{epi}"
            prev = table["choice"].get(key) if args.merge else None
            for c in range(N_CFGS):
                if M > 1024 and c not in BIG_CFGS:  # prefill chunks: the 256x256 kernels or the library
                    continue
                if only_cfgs and c not in only_cfgs and not (prev and prev[0] == c):
                    continue
                bm, bn = hip.gemm_plan.tiles[c]
                tiles = -(-M // bm) * -(-N // bn)
                for sk in SPLITS + ((STREAM_K,) if c == W4_CFG else ()):  # (0 = W4 stream-K)
                    if M > 1024 and sk > 1:
                        continue
                    if only_cfgs and c not in only_cfgs and [c, sk] != list(prev):
                        continue
                    if not hip.gemm_plan.supported(c, M, N, K, epi, sk):
                        continue
                    # split-K: fill the rounds of 256 workgroups; never more than ~8 rounds
                    if sk > 1 and (tiles * sk > 2304 or K // 64 // sk < 6):
                        continue
                    if epi == 2:
                        rr = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
                        got = hip.gemm_nt(x, ws[0], c, 2, residual=rr, out=rr, split_k=sk).float()
                    else:
                        got = hip.gemm_nt(x, ws[0], c, epi, split_k=sk).float()
                    err = (got - ref).abs().max().item() / max(1.0, ref.abs().max().item())
                    if err > 3e-2:
                        print(f"WRONG {proj} M={M} cfg={c} split={sk} err={err}", flush=True)
                        continue
                    if epi == 2:
                        fn = lambda c=c, sk=sk: hip.gemm_nt(x, w_next(), c, 2, residual=r, out=r, split_k=sk)  # noqa
                    else:
                        fn = lambda c=c, sk=sk: hip.gemm_nt(x, w_next(), c, epi, split_k=sk)  # noqa: E731
                    for _ in range(3):
                        fn()
                    res[(c, sk)] = timed(fn, args.reps)
            best = min(res, key=lambda k: res[k] if res[k] is not None else 1e30)
            table["choice"][key] = [-1, 1] if best == "lib" else list(best)
            table["timings_us"][key] = {(k if k == "lib" else f"{k[0]}x{k[1]}"): round(v, 2) for k, v in res.items()}
            hand = min((v for k, v in res.items() if k != "lib"), default=None)
            tf = 2 * M * N * K / (hand * 1e-6) / 1e12 if hand else 0
            print(f"{proj:8s} M={M:4d} N={N:6d} K={K:5d} lib={res['lib']:8.1f}us hand_best={hand:8.1f}us "
                  f"({tf:6.0f} TF/s, x{res['lib'] / hand:4.2f}) -> {table['choice'][key]}  "
                  + " ".join(f"{k[0]}x{k[1]}:{v:.0f}" for k, v in sorted(res.items(), key=lambda kv: kv[1])[:6]
                             if k != "lib"), flush=True)
        del ws
        torch.cuda.empty_cache()
    os.makedirs(os.path.dirname(out_path), exist_ok=True)
    with open(out_path, "w") as fh:
        json.dump(table, fh, indent=1, sort_keys=True)
    print("wrote", out_path)


if __name__ == "__main__":
    main()
