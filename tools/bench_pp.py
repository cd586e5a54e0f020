"""Ping-pong 256x256 GEMM (cfg 10, csrc/kernels/gemm_pp.hip) vs hipBLASLt and the shipped plan.

  python tools/bench_pp.py [--model qwen3-14b] [--m 448,768,16384] [--reps 10]

Per (M, projection): the library path (shipped TunableOp table, same epilogue work
as tools/tune_hand_gemm.py), the current plan choice, and cfg 10 at each split-K,
after a correctness check against F.linear.  Weights rotate over copies that exceed
the 256 MiB Infinity Cache.  Prints one JSON line per shape.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from byzantine_consensus_llm_agents_amd.models.config import ALIASES, get_model_config  # noqa: E402
from byzantine_consensus_llm_agents_amd.ops import get_ops  # noqa: E402
from tools.tune_hand_gemm import shapes, timed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen3-14b")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--m", default="448,768,16384")
    ap.add_argument("--splits", default="1,2,3,4")
    ap.add_argument("--cfgs", default="10,11", help="256x256 kernels to time: 10 ping-pong, 11 four-wave")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    hip = get_ops("hip")
    plan = hip.gemm_plan
    name = ALIASES.get(args.model, args.model).split("/")[-1].lower()
    tuned = os.path.join(ROOT, "byzantine_consensus_llm_agents_amd", "engine", "tuned",
                         f"tunableop_{name}_tp{args.tp}.csv")
    if os.path.exists(tuned):
        t = torch.cuda.tunable
        t.enable(True)
        t.tuning_enable(False)
        t.set_filename(f"/tmp/bcg_bench_pp_{os.getpid()}.csv")
        t.read_file(tuned)
    cfg = get_model_config(args.model)
    gen = torch.Generator(device="cuda").manual_seed(0)
    only = set(filter(None, args.only.split(",")))
    for proj, (N, K, epi) in shapes(cfg, args.tp).items():
        if only and proj not in only:
            continue
        wbytes = N * K * 2
        ws = [torch.randn(N, K, device="cuda", generator=gen).mul_(K ** -0.5).to(torch.bfloat16)
              for _ in range(min(8, max(2, -(-(1 << 30) // wbytes))))]
        for M in [int(m) for m in args.m.split(",")]:
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
                lib = lambda: r.add_(F.linear(x, w_next()))  # noqa: E731
            ref = F.linear(x, ws[0]).float()
            if epi == 1:
                ref = F.silu(ref[:, :N // 2]) * ref[:, N // 2:]
            res = {}
            for _ in range(2):
                lib()
            res["lib"] = timed(lib, args.reps)

            def run(c, sk, w, out_r=None):
                if epi == 2:
                    rr = out_r if out_r is not None else r
                    return hip.gemm_nt(x, w, c, 2, residual=rr, out=rr, split_k=sk)
                return hip.gemm_nt(x, w, c, epi, split_k=sk)

            cands = [(int(c), int(s)) for c in args.cfgs.split(",") for s in args.splits.split(",")]
            choice = plan.choose(M, N, K, epi)
            if choice is not None and choice[0] != 10:
                cands.append(tuple(choice))
            for c, sk in cands:
                if not plan.supported(c, M, N, K, epi, sk):
                    continue
                rr = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16) if epi == 2 else None
                got = run(c, sk, ws[0], rr).float()
                err = (got - ref).abs().max().item() / max(1.0, ref.abs().max().item())
                if err > 3e-2:
                    res[f"{c}x{sk}"] = f"WRONG {err:.3g}"
                    continue
                for _ in range(2):
                    run(c, sk, w_next())
                res[f"{c}x{sk}"] = timed(lambda c=c, sk=sk: run(c, sk, w_next()), args.reps)
            flop = 2 * M * N * K
            best = min((v, k) for k, v in res.items() if isinstance(v, float))
            print(json.dumps({"proj": proj, "M": M, "N": N, "K": K, "epi": epi,
                              "plan": list(choice) if choice else None,
                              "us": {k: (round(v, 1) if isinstance(v, float) else v) for k, v in res.items()},
                              "best": best[1], "best_tflops": round(flop / best[0] / 1e6, 1),
                              "lib_tflops": round(flop / res["lib"] / 1e6, 1)}), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
