"""Which BLAS library path is fastest for the prefill projection GEMMs (what the engine's
library fallback should call).

  python tools/bench_blas_choice.py [--model qwen3-14b] [--m 2048,4096,8192,12288,16384]

Per projection and M (the engine's forms: y = x W^T for qkv / gate_up, r += x W^T via
``residual.addmm_`` for o / down) the median of --reps launches, weights rotated over >= 1 GiB
of copies (no Infinity-Cache hits across launches), for:

  tunable    F.linear / addmm_ with the shipped TunableOp table (what the engine runs today);
  hipblaslt  TunableOp off, hipBLASLt's default heuristic;
  rocblas    TunableOp off, ``preferred_blas_library("cublas")`` (rocBLAS / Tensile).

One JSON line per (projection, M) on stdout.
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from byzantine_consensus_llm_agents_amd.models.config import ALIASES, get_model_config  # noqa: E402


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


def set_mode(mode, table):
    t = torch.cuda.tunable
    if mode == "tunable":
        torch.backends.cuda.preferred_blas_library("cublaslt")
        t.enable(True)
        t.tuning_enable(False)
        t.set_filename(f"/tmp/bcg_blas_choice_{os.getpid()}.csv")
        t.read_file(table)
    else:
        t.enable(False)
        torch.backends.cuda.preferred_blas_library("cublas" if mode == "rocblas" else "cublaslt")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen3-14b")
    ap.add_argument("--m", default="2048,4096,8192,12288,16384")
    ap.add_argument("--modes", default="tunable,hipblaslt,rocblas")
    ap.add_argument("--reps", type=int, default=9)
    args = ap.parse_args()
    cfg = get_model_config(args.model)
    name = ALIASES.get(args.model, args.model).split("/")[-1].lower()
    table = os.path.join(ROOT, "byzantine_consensus_llm_agents_amd", "engine", "tuned", f"tunableop_{name}_tp1.csv")
    H, I, hd = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
    shapes = {"qkv": ((cfg.num_heads + 2 * cfg.num_kv_heads) * hd, H, False), "o": (H, cfg.num_heads * hd, True),
              "gate_up": (2 * I, H, False), "down": (H, I, True)}
    gen = torch.Generator(device="cuda").manual_seed(0)
    for proj, (N, K, resid) in shapes.items():
        copies = max(2, min(8, -(-(1 << 30) // (N * K * 2))))
        ws = [torch.randn(N, K, device="cuda", generator=gen).mul_(K ** -0.5).to(torch.bfloat16) for _ in range(copies)]
        for M in (int(m) for m in args.m.split(",")):
            x = torch.randn(M, K, device="cuda", generator=gen).to(torch.bfloat16)
            r = torch.randn(M, N, device="cuda", generator=gen).to(torch.bfloat16) if resid else None
            it = [0]

            def w_next():
                it[0] = (it[0] + 1) % len(ws)
                return ws[it[0]]

            fn = (lambda: r.addmm_(x, w_next().t())) if resid else (lambda: torch.nn.functional.linear(x, w_next()))
            res = {"proj": proj, "M": M, "N": N, "K": K}
            for mode in args.modes.split(","):
                set_mode(mode, table)
                for _ in range(3):
                    fn()
                us = timed(fn, args.reps)
                res[mode] = round(us, 1)
                res[mode + "_tf"] = round(2 * M * N * K / us / 1e6)
            print(json.dumps(res), flush=True)
            del x, r
        del ws
        torch.cuda.empty_cache()
    set_mode("hipblaslt", table)


if __name__ == "__main__":
    main()
