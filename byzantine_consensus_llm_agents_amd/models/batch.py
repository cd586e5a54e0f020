"""Stand-alone batch builders (paged KV + AttnMeta) for tests, tools and offline scoring.

The engine builds its metadata incrementally (``engine/engine.py``); these
helpers build the same structures for a fixed set of token sequences with
contiguous block assignment, so a model forward can be run without an engine.
"""

from typing import List, Tuple

import torch

from .transformer import AttnMeta, DecoderModel


def alloc_kv(model: DecoderModel, num_blocks: int, block_size: int = 16, device=None, dtype=None):
    dev = device or model.device
    c = model.cfg
    dt = dtype or model.dtype
    k = torch.zeros(c.num_layers, num_blocks, model.n_kv, block_size, model.hd, dtype=dt, device=dev)
    v = torch.zeros(c.num_layers, num_blocks, model.n_kv, model.hd, block_size, dtype=dt, device=dev)
    return k, v


def prefill_batch(seqs: List[List[int]], block_size: int = 16, device="cpu",
                  first_block: int = 1) -> Tuple[torch.Tensor, AttnMeta, int]:
    """Packed prefill of whole sequences; block 0 is left as scratch.

    Returns (tokens [T] int32, meta, number of KV blocks needed)."""
    nblk = [(len(s) + block_size - 1) // block_size for s in seqs]
    width = max(nblk)
    tables = torch.zeros(len(seqs), width, dtype=torch.int32)
    nxt = first_block
    for r, n in enumerate(nblk):
        tables[r, :n] = torch.arange(nxt, nxt + n, dtype=torch.int32)
        nxt += n
    toks, pos, slots, q_start, tiles = [], [], [], [0], []
    for r, s in enumerate(seqs):
        p = torch.arange(len(s))
        toks.extend(s)
        pos.append(p)
        slots.append(tables[r].long()[p // block_size] * block_size + p % block_size)
        for t in range(q_start[-1], q_start[-1] + len(s), 64):
            tiles.append((r, t, min(t + 64, q_start[-1] + len(s))))
        q_start.append(q_start[-1] + len(s))
    i32 = torch.int32
    meta = AttnMeta(
        positions=torch.cat(pos).to(i32).to(device), slots=torch.cat(slots).to(i32).to(device),
        block_tables=tables.to(device), seq_lens=torch.tensor([len(s) for s in seqs], dtype=i32, device=device),
        q_start=torch.tensor(q_start, dtype=i32, device=device), max_q_len=max(len(s) for s in seqs),
        decode=False, logits_idx=torch.tensor([q - 1 for q in q_start[1:]], dtype=torch.int64, device=device),
        tiles=torch.tensor(tiles, dtype=i32, device=device))
    return torch.tensor(toks, dtype=i32, device=device), meta, nxt
