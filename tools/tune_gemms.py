"""Tune the decode-shaped projection GEMMs with PyTorch TunableOp (hipBLASLt + rocBLAS solutions).

  python tools/tune_gemms.py --model qwen3-14b [--tp 1] [--out gpurun_out/tunableop_<model>.csv]

For every decode graph bucket M and every projection of the model (qkv, o,
gate_up, down, lm_head; TP-sharded shapes when --tp > 1), TunableOp times all
candidate solutions and records the fastest.  The CSV is shipped in
byzantine_consensus_llm_agents_amd/engine/tuned/ and loaded by the engine
(lookups only) so the decode graphs use the tuned kernels without tuning at
run time.
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from byzantine_consensus_llm_agents_amd.engine.graphs import BUCKETS  # noqa: E402
from byzantine_consensus_llm_agents_amd.models.config import ALIASES, get_model_config  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="qwen3-14b")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--max-m", type=int, default=512)
    ap.add_argument("--out", default=None)
    ap.add_argument("--extra-m", default="", help="comma list of extra M (e.g. prefill chunk 16384; no lm_head)")
    ap.add_argument("--base", default=None, help="existing TunableOp CSV to extend (results are kept)")
    args = ap.parse_args()
    cfg = get_model_config(args.model)
    name = ALIASES.get(args.model, args.model).split("/")[-1].lower()
    out = args.out or os.path.join(ROOT, "gpurun_out", f"tunableop_{name}_tp{args.tp}.csv")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    tp = args.tp
    H, I, hd = cfg.hidden_size, cfg.intermediate_size // tp, cfg.head_dim
    nq, nkv = cfg.num_heads // tp, cfg.num_kv_heads // tp
    shapes = {"qkv": ((nq + 2 * nkv) * hd, H), "o": (H, nq * hd), "gate_up": (2 * I, H), "down": (H, I),
              "lm_head": (cfg.vocab_size // tp, H)}
    torch.cuda.tunable.enable(True)
    torch.cuda.tunable.tuning_enable(True)
    torch.cuda.tunable.set_max_tuning_duration(40)
    torch.cuda.tunable.set_filename(out)
    if args.base and os.path.exists(args.base):
        torch.cuda.tunable.read_file(args.base)
    ws = {k: torch.randn(n, kk, device="cuda", dtype=torch.bfloat16) for k, (n, kk) in shapes.items()}
    t0 = time.time()
    extra = [int(m) for m in args.extra_m.split(",") if m]
    for M in [b for b in BUCKETS if b <= args.max_m] + extra:
        for k, w in ws.items():
            if M > 4096 and k == "lm_head":
                continue  # prefill computes logits for the last token of each sequence only
            x = torch.randn(M, w.shape[1], device="cuda", dtype=torch.bfloat16)
            torch.nn.functional.linear(x, w)
        torch.cuda.synchronize()
        print(f"M={M} tuned ({time.time() - t0:.0f}s)", flush=True)
    torch.cuda.tunable.tuning_enable(False)
    res = torch.cuda.tunable.get_results()
    print(f"{len(res)} results -> {out}")


if __name__ == "__main__":
    main()
