"""PyTorch reference implementations of every engine op (fp32 math).

These define the semantics the HIP kernels in ``csrc/kernels`` must match and
run the ``torch`` backend (CPU tests).  Layout conventions shared with the
kernels:

* KV cache: ``k_cache : [L, num_blocks, n_kv, block_size, head_dim]`` and
  ``v_cache : [L, num_blocks, n_kv, head_dim, block_size]`` (V stored
  transposed per block-head: it is the A operand of ``O^T = V^T P^T`` in the
  MFMA attention kernels); bf16; block 0 is a never-allocated scratch block.
* ``block_tables : [B, max_blocks] int32``; ``seq_lens : [B] int32`` = number
  of tokens whose KV is resident *including* the tokens of this step.
* Sampling: Gumbel-max with a counter-based hash (``gumbel_hash``) so the
  HIP kernel and this reference pick identical tokens from identical logits.
"""

import math
from typing import Optional, Tuple

import torch

MASK32 = 0xFFFFFFFF


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
    return y.to(x.dtype)


def add_rmsnorm(x: torch.Tensor, residual: Optional[torch.Tensor], w: torch.Tensor,
                eps: float) -> Tuple[torch.Tensor, torch.Tensor]:
    """``residual <- residual + x`` (in place, or x itself if None); returns (norm(residual), residual)."""
    if residual is None:
        residual = x.clone()
    else:
        residual.copy_((residual.float() + x.float()).to(residual.dtype))
    return rmsnorm(residual, w, eps), residual


def embed_rmsnorm(tokens: torch.Tensor, table: torch.Tensor, w: torch.Tensor,
                  eps: float) -> Tuple[torch.Tensor, torch.Tensor]:
    """Embedding gather fused with the first RMSNorm: (rmsnorm(E[tokens]) * w, E[tokens])."""
    residual = table.index_select(0, tokens.long())
    return rmsnorm(residual, w, eps), residual


def rope_cache(max_pos: int, head_dim: int, theta: float, device=None) -> torch.Tensor:
    """[max_pos, head_dim] fp32: first half cos, second half sin (neox layout)."""
    half = head_dim // 2
    inv = 1.0 / (theta ** (torch.arange(0, half, dtype=torch.float64) * 2 / head_dim))
    ang = torch.arange(max_pos, dtype=torch.float64)[:, None] * inv[None, :]
    return torch.cat([ang.cos(), ang.sin()], dim=-1).float().to(device)


def _rope(x: torch.Tensor, cs: torch.Tensor) -> torch.Tensor:
    half = x.shape[-1] // 2
    cos, sin = cs[..., :half], cs[..., half:]
    x1, x2 = x[..., :half], x[..., half:]
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1)


def qk_norm_rope_kv_write(qkv: torch.Tensor, positions: torch.Tensor, slots: torch.Tensor,
                          n_q: int, n_kv: int, head_dim: int, q_norm: Optional[torch.Tensor],
                          k_norm: Optional[torch.Tensor], eps: float, cos_sin: torch.Tensor,
                          k_cache: torch.Tensor, v_cache: torch.Tensor, layer: int,
                          contiguous: bool = True) -> torch.Tensor:
    """Split fused QKV, (Qwen3) RMSNorm q/k per head, neox RoPE, scatter K/V into the paged cache.

    Returns q as ``[T, n_q, head_dim]`` (activation dtype).
    """
    T = qkv.shape[0]
    q = qkv[:, : n_q * head_dim].float().view(T, n_q, head_dim)
    k = qkv[:, n_q * head_dim:(n_q + n_kv) * head_dim].float().view(T, n_kv, head_dim)
    v = qkv[:, (n_q + n_kv) * head_dim:].view(T, n_kv, head_dim)
    if q_norm is not None:
        q = q * torch.rsqrt(q.pow(2).mean(-1, keepdim=True) + eps) * q_norm.float()
        k = k * torch.rsqrt(k.pow(2).mean(-1, keepdim=True) + eps) * k_norm.float()
    cs = cos_sin[positions.long()][:, None, :]
    q = _rope(q, cs)
    k = _rope(k, cs)
    bs = k_cache.shape[3]
    blk = (slots // bs).long()
    off = (slots % bs).long()
    if k_cache.dtype == torch.float8_e4m3fn:  # fp8 KV cache: saturate (e4m3fn has no inf)
        k, v = k.clamp(-448.0, 448.0), v.float().clamp(-448.0, 448.0)
    k_cache[layer, blk, :, off] = k.to(k_cache.dtype)
    v_cache[layer, blk, :, :, off] = v.to(v_cache.dtype)
    return q.to(qkv.dtype)


def _gather_kv(cache, layer, table_row, ctx, transposed=False):
    blocks = cache[layer]
    if transposed:                                        # V: [NB, n_kv, hd, bs]
        blocks = blocks.transpose(2, 3)
    bs = blocks.shape[2]
    nblk = (ctx + bs - 1) // bs
    sel = blocks[table_row[:nblk].long()]                  # [nblk, n_kv, bs, hd]
    return sel.permute(1, 0, 2, 3).reshape(sel.shape[1], nblk * bs, sel.shape[3])[:, :ctx]


def paged_attention(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, layer: int,
                    block_tables: torch.Tensor, q_start: torch.Tensor, seq_lens: torch.Tensor,
                    scale: float) -> torch.Tensor:
    """Causal GQA attention of packed queries over paged KV.

    ``q : [T, n_q, hd]``; sequence b owns query rows ``q_start[b]:q_start[b+1]``
    which are its LAST rows, i.e. positions ``seq_lens[b]-q_len .. seq_lens[b]-1``.
    Returns ``[T, n_q*hd]``.
    """
    T, n_q, hd = q.shape
    n_kv = k_cache.shape[2]
    group = n_q // n_kv
    out = torch.zeros(T, n_q, hd, dtype=torch.float32, device=q.device)
    for b in range(block_tables.shape[0]):
        s, e = int(q_start[b]), int(q_start[b + 1])
        if e <= s:
            continue
        ctx = int(seq_lens[b])
        k = _gather_kv(k_cache, layer, block_tables[b], ctx).float()   # [n_kv, ctx, hd]
        v = _gather_kv(v_cache, layer, block_tables[b], ctx, transposed=True).float()
        k = k.repeat_interleave(group, 0)
        v = v.repeat_interleave(group, 0)
        qb = q[s:e].float().permute(1, 0, 2)                            # [n_q, qlen, hd]
        scores = torch.matmul(qb, k.transpose(1, 2)) * scale            # [n_q, qlen, ctx]
        qpos = torch.arange(ctx - (e - s), ctx, device=q.device)[:, None]
        kpos = torch.arange(ctx, device=q.device)[None, :]
        scores = scores.masked_fill(kpos > qpos, float("-inf"))
        out[s:e] = torch.matmul(torch.softmax(scores, -1), v).permute(1, 0, 2)
    return out.reshape(T, n_q * hd).to(q.dtype)


def _partial(q, k, v, scale):
    """(O unnormalised, m, l) of q [n_q, hd] over k, v [n_q, n, hd] -- one flash-decoding split."""
    s = torch.einsum("hd,hnd->hn", q, k) * scale
    m = s.max(-1).values
    p = torch.exp(s - m[:, None])
    return torch.einsum("hn,hnd->hd", p, v), m, p.sum(-1)


def paged_attention_decode_cascade(q, k_cache, v_cache, layer, block_tables, seq_lens, scale, cascade):
    """Decode attention the way the HIP cascade computes it, from its tables (fp32).

    A grouped row's tokens [0, kv_begin) come from its group's FIRST member's block table
    (``decode_shared_kernel``, in pieces -- merged here as one); [kv_begin, ctx) from its own
    (``decode_attn_kernel``); the partials merge as flash-decoding splits do.  Equal to
    `paged_attention` exactly when the tables are consistent (every member holds the group's
    block ids) -- what the CPU tests of ``engine/cascade.py`` check.  ``cascade``: CascadeTables (any device)."""
    B, n_q, hd = q.shape
    n_kv = k_cache.shape[2]
    group = n_q // n_kv
    kv_begin = cascade.kv_begin.cpu().tolist()
    lead_of = {}
    desc = cascade.grp_desc.cpu().tolist()
    rows = cascade.grp_rows.cpu().tolist()
    items = cascade.items.cpu().tolist()[:int(cascade.n_items[0])]
    for g, _, _, _ in items:
        first, n, shared = desc[g][:3]
        for m in rows[first:first + n]:
            lead_of[m] = (rows[first], shared * k_cache.shape[3])
    out = torch.zeros(B, n_q, hd, dtype=torch.float32)
    for b in range(B):
        ctx = int(seq_lens[b])
        qb = q[b].float().cpu()
        parts = []
        begin = kv_begin[b]
        if begin:
            lead, shared = lead_of[b]
            assert shared == begin, "kv_begin disagrees with the group table"
            k = _gather_kv(k_cache, layer, block_tables[lead], shared).float().cpu().repeat_interleave(group, 0)
            v = _gather_kv(v_cache, layer, block_tables[lead], shared, True).float().cpu().repeat_interleave(group, 0)
            parts.append(_partial(qb, k, v, scale))
        k = _gather_kv(k_cache, layer, block_tables[b], ctx).float().cpu()[:, begin:].repeat_interleave(group, 0)
        v = _gather_kv(v_cache, layer, block_tables[b], ctx, True).float().cpu()[:, begin:].repeat_interleave(group, 0)
        parts.append(_partial(qb, k, v, scale))
        m = torch.stack([p[1] for p in parts]).max(0).values
        o = sum(p[0] * torch.exp(p[1] - m)[:, None] for p in parts)
        l_sum = sum(p[2] * torch.exp(p[1] - m) for p in parts)
        out[b] = o / l_sum[:, None]
    return out.reshape(B, n_q * hd).to(q.dtype)


def linear_silu(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """silu(x Wg^T) * (x Wu^T) with W = [gate; up]: the fused gate_up GEMM epilogue (fp32 math)."""
    gu = x.float() @ w.float().t()
    inter = gu.shape[-1] // 2
    return (torch.nn.functional.silu(gu[:, :inter]) * gu[:, inter:]).to(x.dtype)


def linear_residual(x: torch.Tensor, w: torch.Tensor, residual: torch.Tensor) -> torch.Tensor:
    """residual <- residual + x W^T, rounded once (the fused o/down GEMM epilogue); in place."""
    residual.copy_((residual.float() + x.float() @ w.float().t()).to(residual.dtype))
    return residual


def silu_mul(gu: torch.Tensor) -> torch.Tensor:
    inter = gu.shape[-1] // 2
    g, u = gu[..., :inter].float(), gu[..., inter:].float()
    return (g * torch.sigmoid(g) * u).to(gu.dtype)


# ------------------------------------------------------------------ sampling
def _fmix32(h: torch.Tensor) -> torch.Tensor:
    h = h & MASK32
    h = h ^ (h >> 16)
    h = (h * 0x85EBCA6B) & MASK32
    h = h ^ (h >> 13)
    h = (h * 0xC2B2AE35) & MASK32
    return h ^ (h >> 16)


def gumbel_hash(seed: int, row_key: torch.Tensor, step: int, tokens: torch.Tensor) -> torch.Tensor:
    """Uniform (0,1) from (seed, row key, step, token) -- same bits as sample.hip."""
    a = _fmix32((row_key.long() * 0x9E3779B9 + step * 0x632BE5AB + seed) & MASK32)
    h = _fmix32(a[:, None] ^ ((tokens.long()[None, :] * 0x27D4EB2F) & MASK32))
    return ((h >> 8).double() + 0.5) / 16777216.0


def sample_step(logits: torch.Tensor, fsm_next: torch.Tensor, fsm_dist: torch.Tensor,
                fsm_base: torch.Tensor, fsm_state: torch.Tensor, gen_count: torch.Tensor,
                max_new: torch.Tensor, temperature: torch.Tensor, row_keys: torch.Tensor,
                done: torch.Tensor, seq_lens: torch.Tensor, out_tokens: torch.Tensor,
                next_tokens: torch.Tensor, seed: int, budget_aware: bool, n_text_tokens: int,
                eos_id: int, eos_id2: int) -> None:
    """One guided sampling step for every row, updating all per-row state in place.

    Row b is guided when ``fsm_base[b] >= 0`` (allowed tokens: those with
    ``fsm_next[base+state, t] >= 0``; in budget mode additionally
    ``fsm_dist[base+next] <= remaining-1`` whenever some token satisfies it);
    otherwise every text token and the EOS ids are allowed.  The sampled token
    goes to ``out_tokens[b, gen_count[b]]`` and ``next_tokens[b]``;
    ``gen_count`` and ``seq_lens`` advance.  Rows already ``done`` are untouched.
    """
    B, V = logits.shape
    tok_ids = torch.arange(V, device=logits.device)
    for b in range(B):
        if bool(done[b]):
            continue
        base = int(fsm_base[b])
        step = int(gen_count[b])
        rem = int(max_new[b]) - step
        lg = logits[b].float()
        if base >= 0:
            row = base + int(fsm_state[b])
            nxt = fsm_next[row, :V].long()
            ok = nxt >= 0
            if budget_aware:
                dist_next = torch.where(ok, fsm_dist[(base + nxt.clamp(min=0))].long(),
                                        torch.full_like(nxt, 1 << 20))
                tight = ok & (dist_next <= rem - 1)
                if bool(tight.any()):
                    ok = tight
        else:
            ok = (tok_ids < n_text_tokens) | (tok_ids == eos_id) | (tok_ids == eos_id2)
        if not bool(ok.any()):
            done[b] = 1
            continue
        t = float(temperature[b])
        if t <= 0:
            score = lg.double()
        else:
            u = gumbel_hash(seed, row_keys[b:b + 1], step, tok_ids)[0]
            score = lg.double() / t - torch.log(-torch.log(u))
        score = torch.where(ok, score, torch.full_like(score, -math.inf))
        tok = int(torch.argmax(score))
        out_tokens[b, step] = tok
        next_tokens[b] = tok
        gen_count[b] = step + 1
        seq_lens[b] += 1
        finished = rem - 1 <= 0
        if base >= 0:
            ns = int(fsm_next[base + int(fsm_state[b]), tok])
            fsm_state[b] = ns
            finished = finished or int(fsm_dist[base + ns]) == 0
        else:
            finished = finished or tok in (eos_id, eos_id2)
        if finished:
            done[b] = 1


# ------------------------------------------------------------------ fp8 (OCP e4m3fn)
FP8_MAX = 448.0
FP8 = torch.float8_e4m3fn


def quant_fp8(x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Row-wise dynamic quantisation: scale = max|x_row| / 448, q = x / scale (fp8 e4m3fn)."""
    xf = x.float()
    scale = xf.abs().amax(dim=-1).clamp(min=1e-12) / FP8_MAX
    q = (xf / scale[:, None]).clamp(-FP8_MAX, FP8_MAX).to(FP8)
    return q, scale


def add_rmsnorm_fp8(x, residual, w, eps):
    """add_rmsnorm (bf16-rounded output, as the bf16 path) then row-wise fp8 quantisation."""
    y, residual = add_rmsnorm(x, residual, w, eps)
    q, s = quant_fp8(y)
    return q, s, residual


def rmsnorm_fp8(x, w, eps):
    """Plain RMSNorm (bf16-rounded, as the bf16 path) then row-wise fp8 quantisation."""
    return quant_fp8(rmsnorm(x, w, eps))


def embed_rmsnorm_fp8(tokens, table, w, eps):
    """(fp8(rmsnorm(table[tokens]) * w), row scales, table[tokens])."""
    y, residual = embed_rmsnorm(tokens, table, w, eps)
    q, s = quant_fp8(y)
    return q, s, residual


def linear_fp8_residual(xq, xs, wq, ws, residual):
    """residual <- residual + dequant(xq . wq^T), rounded once (the fused fp8 epilogue); in place."""
    y = (xq.float() * xs[:, None]) @ (wq.float() * ws[:, None]).t()
    residual.copy_((residual.float() + y).to(residual.dtype))
    return residual


def silu_mul_fp8(gu):
    return quant_fp8(silu_mul(gu))


def quantize_weight_fp8(w: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-output-channel weight quantisation: w [N, K] -> (fp8 [N, K], scale fp32 [N])."""
    return quant_fp8(w)


def linear_fp8(xq, xs, wq, ws, bias=None, out_dtype=torch.bfloat16):
    """y = (xq * xs[:, None]) @ (wq * ws[:, None])^T (+ bias), fp32 accumulate."""
    y = (xq.float() * xs[:, None]) @ (wq.float() * ws[:, None]).t()
    if bias is not None:
        y = y + bias.float()
    return y.to(out_dtype)
