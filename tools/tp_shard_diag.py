"""Kernel check of ONE TP rank's shard shapes on one GPU (no collectives): the HIP forward of
rank r's shard (bf16) against the fp32 torch forward of the same shard, with a stub TP group
whose all-reduce is the identity (both sides then compute the same partial sums).  Localises a
TP mismatch to the per-rank kernels (GEMM table entries at shard shapes, attention at the
shard's head counts) or, if this agrees, to the collectives.

usage: python tools/tp_shard_diag.py MODEL TP [LAYERS] [fp8]
"""
import dataclasses
import sys

import torch

sys.path.insert(0, ".")
from byzantine_consensus_llm_agents_amd.models.config import get_model_config  # noqa: E402
from byzantine_consensus_llm_agents_amd.models.transformer import AttnMeta, DecoderModel, TPGroup  # noqa: E402
from byzantine_consensus_llm_agents_amd.ops import get_ops  # noqa: E402


class StubTP(TPGroup):
    def all_reduce_(self, x):
        return x

    def all_reduce_add_rmsnorm(self, x, residual, w, eps, ops):
        return ops.add_rmsnorm(x, residual, w, eps)

    def all_gather_last(self, x):
        return torch.cat([x] * self.size, dim=-1)


def main():
    name, tp = sys.argv[1], int(sys.argv[2])
    layers = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    quant = "fp8" if "fp8" in sys.argv[4:] else None
    cfg = dataclasses.replace(get_model_config(name), num_layers=layers)
    g = StubTP(None, 0, tp)
    mh = DecoderModel(cfg, get_ops("hip"), "cuda", torch.bfloat16, g, quant=quant)
    mh.init_random(seed=7, std=0.02)
    mt = DecoderModel(cfg, get_ops("torch"), "cuda", torch.float32, g, quant=quant)
    mt.layers = [{k: (v.float() if v.dtype == torch.bfloat16 else v) for k, v in L.items()} for L in mh.layers]
    mt.embed, mt.lm_head, mt.final_norm = mh.embed.float(), mh.lm_head.float(), mh.final_norm.float()
    mt.cos_sin = mh.cos_sin
    LENS, BS = [37, 150, 301, 64, 90, 411, 16, 222], 16
    B = len(LENS)
    nb = (max(LENS) + 8 + BS - 1) // BS
    tables = (torch.arange(B * nb, dtype=torch.int32) + 1).view(B, nb)
    caches = []
    for m, dt in ((mh, torch.bfloat16), (mt, torch.float32)):
        caches.append((torch.zeros(layers, B * nb + 1, m.n_kv, BS, m.hd, dtype=dt, device="cuda"),
                       torch.zeros(layers, B * nb + 1, m.n_kv, m.hd, BS, dtype=dt, device="cuda")))
    gen = torch.Generator().manual_seed(11)
    toks, pos, slots, q_start, tiles = [], [], [], [0], []
    for r, n in enumerate(LENS):
        toks += torch.randint(0, min(cfg.vocab_size, 30000), (n,), generator=gen).tolist()
        p = torch.arange(n)
        pos.append(p)
        slots.append(tables[r].long()[p // BS] * BS + p % BS)
        for t in range(q_start[-1], q_start[-1] + n, 64):
            tiles.append((r, t, min(t + 64, q_start[-1] + n)))
        q_start.append(q_start[-1] + n)
    i32 = torch.int32
    meta = AttnMeta(positions=torch.cat(pos).to(i32).cuda(), slots=torch.cat(slots).to(i32).cuda(),
                    block_tables=tables.cuda(), seq_lens=torch.tensor(LENS, dtype=i32).cuda(),
                    q_start=torch.tensor(q_start, dtype=i32).cuda(), max_q_len=max(LENS),
                    logits_idx=torch.tensor([q - 1 for q in q_start[1:]]).cuda(),
                    tiles=torch.tensor(tiles, dtype=i32).cuda())
    tok = torch.tensor(toks, dtype=i32).cuda()
    outs = [m.forward(tok, meta, *c).float() for m, c in ((mh, caches[0]), (mt, caches[1]))]
    V = mh.vocab_local
    a, b = outs[0][:, :V], outs[1][:, :V]
    cos = torch.nn.functional.cosine_similarity(a, b, dim=-1)
    print(f"[shard] {name} tp={tp} layers={layers} quant={quant} prefill: min cos {cos.min().item():.5f} "
          f"n_q={mh.n_q} n_kv={mh.n_kv} inter={mh.inter} V_local={V}")
    p = torch.tensor(LENS)
    dmeta = AttnMeta(positions=p.to(i32).cuda(), slots=(tables[torch.arange(B), p // BS].long() * BS + p % BS).to(i32).cuda(),
                     block_tables=tables.cuda(), seq_lens=(p + 1).to(i32).cuda(), decode=True)
    nxt = a.argmax(-1).to(i32)
    outs = [m.forward(nxt, dmeta, *c).float() for m, c in ((mh, caches[0]), (mt, caches[1]))]
    cos = torch.nn.functional.cosine_similarity(outs[0][:, :V], outs[1][:, :V], dim=-1)
    print(f"[shard] {name} tp={tp} decode: min cos {cos.min().item():.5f}")


if __name__ == "__main__":
    main()
