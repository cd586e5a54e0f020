"""Tensor-parallel decoder (Qwen3 / Qwen2 / Mistral) over paged KV.

One forward serves both phases:

* prefill - packed variable-length prompts (``T = sum of uncached prompt
  tokens``), attention over cached prefix + new tokens;
* decode  - one token per sequence (``T = B``), captured into a HIP graph by
  the engine.

Per layer: fused residual-add+RMSNorm -> QKV GEMM -> fused
QK-norm+RoPE+paged-KV-write (HIP) -> paged attention (HIP, MFMA) -> o_proj GEMM
[-> all-reduce fused with the next add+RMSNorm] -> gate_up GEMM with SiLU*mul in its
epilogue -> down GEMM [-> all-reduce fused with the next add+RMSNorm]; at TP=1 the
residual adds ride in the o/down GEMM epilogues.  Column-parallel
QKV/gate_up, row-parallel o/down, vocab-parallel LM head + all-gather, so a
TP group does 2L+1 collectives per forward like the reference's vLLM path.
"""

from dataclasses import dataclass
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

from .config import ModelConfig


@dataclass
class AttnMeta:
    """Attention inputs of one forward (all device tensors)."""

    positions: torch.Tensor      # [T] int32
    slots: torch.Tensor          # [T] int32 (physical KV slot of each new token)
    block_tables: torch.Tensor   # [B, max_blocks] int32
    seq_lens: torch.Tensor       # [B] int32, tokens resident after this step
    q_start: Optional[torch.Tensor] = None   # [B+1] int32 (prefill only)
    max_q_len: int = 1
    decode: bool = False
    logits_idx: Optional[torch.Tensor] = None  # rows whose logits are needed
    tiles: Optional[torch.Tensor] = None       # [n_tiles, 3] int32 prefill work list (HIP kernel)
    tile_rows: int = 64                        # rows per `tiles` entry (ops.prefill_tile_rows)
    workspace: Optional[torch.Tensor] = None   # decode split-K scratch shared by all graphs (HIP)
    cascade: Optional[object] = None           # decode shared-prefix tables (engine/cascade.py)
    # decode: the context lengths the attention reads (None = seq_lens).  The engine gives rows
    # that already finished (they idle in the batch until the host reaps them) one token, so
    # their KV is not streamed again every step; their outputs are ignored by the sampler
    attn_seq_lens: Optional[torch.Tensor] = None


class TPGroup:
    """Thin wrapper over a torch.distributed process group (RCCL on ROCm).

    ``custom`` (optional): an xGMI peer-memory all-reduce
    (``parallel.custom_allreduce.XGMIAllReduce``) used for every message it
    accepts -- the decode-sized ones; the rest go through RCCL.
    ``chunk_large``: messages beyond the custom kernel's cap go through it in cap-sized
    pieces instead of the process group -- set when that group is gloo (ranks sharing one
    GPU: a gloo all-reduce of a prefill chunk is a host round trip per call).
    """

    def __init__(self, group=None, rank: int = 0, size: int = 1, custom=None, ctrl=None, leader: int = 0,
                 chunk_large: bool = False):
        self.group, self.rank, self.size, self.custom = group, rank, size, custom
        self.ctrl = ctrl        # CPU (gloo) group of the same ranks: the driver's plan broadcasts
        # "on" (xGMI kernels, cross-checked), "off" (not requested) or "fallback:<reason>"
        self.custom_status = "on" if custom is not None else "off"
        self.leader = leader    # global rank of this group's rank 0 (the driver)
        self.chunk_large = chunk_large

    def _chunkable(self, x: torch.Tensor) -> bool:
        return (self.chunk_large and self.custom is not None and x.dtype == torch.bfloat16
                and x.is_contiguous() and x.numel() % 8 == 0)

    def all_reduce_(self, x: torch.Tensor) -> torch.Tensor:
        if self.size > 1:
            if self.custom is not None and self.custom.can(x):
                self.custom.all_reduce_(x)
            elif self._chunkable(x):
                flat, step = x.view(-1), (self.custom.cap_bytes // 2) // 8 * 8
                for i in range(0, flat.numel(), step):
                    self.custom.all_reduce_(flat[i:i + step])
            else:
                torch.distributed.all_reduce(x, group=self.group)
        return x

    def all_reduce_add_rmsnorm(self, x: torch.Tensor, residual: Optional[torch.Tensor], w: torch.Tensor,
                               eps: float, ops):
        """(rmsnorm(residual + sum_ranks x) * w, updated residual): the row-parallel projection's
        all-reduce fused with the next residual add + RMSNorm where the xGMI kernel takes it."""
        if self.size > 1 and residual is not None and self.custom is not None and x.is_cuda:
            if self.custom.can_addnorm(x):
                return self.custom.all_reduce_add_rmsnorm(x, residual, w, eps), residual
            if x.dim() == 2 and self._chunkable(x) and residual.is_contiguous():
                rows = max(1, self.custom.cap_bytes // (2 * x.shape[1]))
                if self.custom.can_addnorm(x[:rows]):
                    h = torch.cat([self.custom.all_reduce_add_rmsnorm(x[r:r + rows], residual[r:r + rows], w, eps)
                                   for r in range(0, x.shape[0], rows)])
                    return h, residual
        return ops.add_rmsnorm(self.all_reduce_(x), residual, w, eps)

    def all_gather_last(self, x: torch.Tensor) -> torch.Tensor:
        if self.size == 1:
            return x
        x = x.contiguous()
        full_shape = x.shape[:-1] + (x.shape[-1] * self.size,)
        if self.custom is not None and x.is_cuda and x.dtype == torch.bfloat16:
            # small gathers (decode logits of a few rows) over the xGMI kernel: every rank
            # places its shard in a zeroed full-width tensor and the shards are summed --
            # exact (x + 0), graph-capturable, no RCCL call inside a captured decode step
            # (beyond the kernel's cap: in pieces when the group is gloo -- graph capture
            # cannot hold a gloo collective)
            full = torch.zeros(full_shape, dtype=x.dtype, device=x.device)
            if self.custom.can(full) or self._chunkable(full):
                w_ = x.shape[-1]
                full[..., self.rank * w_:(self.rank + 1) * w_].copy_(x)
                return self.all_reduce_(full)
        parts = [torch.empty_like(x) for _ in range(self.size)]
        torch.distributed.all_gather(parts, x, group=self.group)
        return torch.cat(parts, dim=-1)


class DecoderModel:
    PROJECTIONS = ("qkv", "o", "gate_up", "down")

    def __init__(self, cfg: ModelConfig, ops, device, dtype=torch.bfloat16,
                 tp: Optional[TPGroup] = None, quant: Optional[str] = None):
        if quant not in (None, "fp8"):
            raise ValueError(f"unsupported quantization {quant!r} (None or 'fp8')")
        self.quant = quant
        self.cfg = cfg
        self.ops = ops
        self.device = torch.device(device)
        self.dtype = dtype
        self.tp = tp or TPGroup()
        ts = self.tp.size
        if cfg.num_heads % ts or cfg.num_kv_heads % ts or cfg.intermediate_size % ts or cfg.vocab_size % ts:
            raise ValueError(f"{cfg.name}: heads/intermediate/vocab not divisible by tp={ts}")
        self.n_q = cfg.num_heads // ts
        self.n_kv = cfg.num_kv_heads // ts
        self.inter = cfg.intermediate_size // ts
        self.vocab_local = cfg.vocab_size // ts
        self.hd = cfg.head_dim
        self.scale = cfg.head_dim ** -0.5
        self.layers: List[Dict[str, torch.Tensor]] = []
        self.embed: Optional[torch.Tensor] = None
        self.lm_head: Optional[torch.Tensor] = None
        self.final_norm: Optional[torch.Tensor] = None
        self.cos_sin = None

    # ------------------------------------------------------------- weights
    def _shapes(self):
        c, h = self.cfg, self.cfg.hidden_size
        qkv_out = (self.n_q + 2 * self.n_kv) * self.hd
        shapes = {"qkv": (qkv_out, h), "o": (h, self.n_q * self.hd), "gate_up": (2 * self.inter, h),
                  "down": (h, self.inter), "ln1": (h,), "ln2": (h,)}
        if c.qkv_bias:
            shapes["qkv_bias"] = (qkv_out,)
        if c.qk_norm:
            shapes["q_norm"] = (self.hd,)
            shapes["k_norm"] = (self.hd,)
        return shapes

    def init_random(self, seed: int = 0, std: float = 0.02):
        """Random-init weights, identical for every TP degree.

        Each full (unsharded) tensor is drawn from its own seeded generator and
        then sliced exactly like a checkpoint (`_load_layer`), so a TP=2 engine
        holds the two halves of the TP=1 engine's weights (TP-vs-TP=1 parity
        tests, and every rank derives its shard without communication).
        """
        c, hd, H = self.cfg, self.hd, self.cfg.hidden_size
        gen = torch.Generator(device=self.device)

        def normal(shape, tag):
            gen.manual_seed((seed * 1000003 + tag * 7919 + 17) & 0x7FFFFFFFFFFFFFFF)
            t = torch.empty(*shape, device=self.device, dtype=self.dtype)
            t.normal_(0.0, std, generator=gen)
            return t

        def ones(n):
            return torch.ones(n, device=self.device, dtype=self.dtype)

        full = {"self_attn.q_proj.weight": (c.num_heads * hd, H), "self_attn.k_proj.weight": (c.num_kv_heads * hd, H),
                "self_attn.v_proj.weight": (c.num_kv_heads * hd, H), "self_attn.o_proj.weight": (H, c.num_heads * hd),
                "mlp.gate_proj.weight": (c.intermediate_size, H), "mlp.up_proj.weight": (c.intermediate_size, H),
                "mlp.down_proj.weight": (H, c.intermediate_size)}
        if c.qkv_bias:
            full.update({"self_attn.q_proj.bias": (c.num_heads * hd,), "self_attn.k_proj.bias": (c.num_kv_heads * hd,),
                         "self_attn.v_proj.bias": (c.num_kv_heads * hd,)})
        self.layers = []
        for i in range(c.num_layers):
            tensors = {name: normal(shape, 64 * i + j) for j, (name, shape) in enumerate(full.items())}
            tensors["input_layernorm.weight"] = ones(H)
            tensors["post_attention_layernorm.weight"] = ones(H)
            if c.qk_norm:
                tensors["self_attn.q_norm.weight"] = ones(hd)
                tensors["self_attn.k_norm.weight"] = ones(hd)
            self.layers.append(self._load_layer(tensors.__getitem__))
            del tensors
        self.embed = normal((c.vocab_size, H), 1 << 20)
        if c.tie_embeddings:
            lo = self.tp.rank * self.vocab_local
            self.lm_head = self.embed[lo:lo + self.vocab_local]
        else:
            head = normal((c.vocab_size, H), (1 << 20) + 1)
            lo = self.tp.rank * self.vocab_local
            self.lm_head = head[lo:lo + self.vocab_local].contiguous()
            del head
        self.final_norm = ones(H)
        self._finish()

    def _load_layer(self, get) -> Dict[str, torch.Tensor]:
        """This rank's shard of one decoder layer from HF-named full tensors (`get(name)`):
        column-parallel q/k/v and gate/up (row blocks), row-parallel o/down (column blocks)."""
        c, r, hd = self.cfg, self.tp.rank, self.hd

        def rows(t, n_local, per=1):
            return t[r * n_local * per:(r + 1) * n_local * per]

        q = rows(get("self_attn.q_proj.weight"), self.n_q, hd)
        k = rows(get("self_attn.k_proj.weight"), self.n_kv, hd)
        v = rows(get("self_attn.v_proj.weight"), self.n_kv, hd)
        layer = {"qkv": torch.cat([q, k, v]).contiguous(),
                 "o": get("self_attn.o_proj.weight")[:, r * self.n_q * hd:(r + 1) * self.n_q * hd].contiguous(),
                 "gate_up": torch.cat([rows(get("mlp.gate_proj.weight"), self.inter),
                                       rows(get("mlp.up_proj.weight"), self.inter)]).contiguous(),
                 "down": get("mlp.down_proj.weight")[:, r * self.inter:(r + 1) * self.inter].contiguous(),
                 "ln1": get("input_layernorm.weight"),
                 "ln2": get("post_attention_layernorm.weight")}
        if c.qkv_bias:
            layer["qkv_bias"] = torch.cat([rows(get("self_attn.q_proj.bias"), self.n_q, hd),
                                           rows(get("self_attn.k_proj.bias"), self.n_kv, hd),
                                           rows(get("self_attn.v_proj.bias"), self.n_kv, hd)])
        if c.qk_norm:
            layer["q_norm"] = get("self_attn.q_norm.weight")
            layer["k_norm"] = get("self_attn.k_norm.weight")
        return layer

    def load_hf_state_dict(self, sd: Dict[str, torch.Tensor]):
        """Load (and TP-slice) an HF-named state dict (Qwen2/Qwen3/Mistral naming)."""
        c = self.cfg

        def get(name):
            return sd[name].to(device=self.device, dtype=self.dtype)

        self.layers = [self._load_layer(lambda n, p=f"model.layers.{i}.": get(p + n)) for i in range(c.num_layers)]
        self.embed = get("model.embed_tokens.weight")
        head = self.embed if c.tie_embeddings or "lm_head.weight" not in sd else get("lm_head.weight")
        lo = self.tp.rank * self.vocab_local
        self.lm_head = head[lo:lo + self.vocab_local].contiguous()
        self.final_norm = get("model.norm.weight")
        self._finish()

    def hf_state_dict(self) -> Dict[str, torch.Tensor]:
        """HF-named full state dict (TP=1 only): inverse of `load_hf_state_dict`."""
        if self.tp.size != 1 or self.quant:
            raise ValueError("hf_state_dict exports unsharded, unquantised weights (tp=1, bf16)")
        c, hd = self.cfg, self.hd
        nq, nkv = self.n_q * hd, self.n_kv * hd
        sd = {}
        for i, L in enumerate(self.layers):
            p = f"model.layers.{i}."
            q, k, v = L["qkv"].split([nq, nkv, nkv])
            sd[p + "self_attn.q_proj.weight"], sd[p + "self_attn.k_proj.weight"] = q, k
            sd[p + "self_attn.v_proj.weight"] = v
            sd[p + "self_attn.o_proj.weight"] = L["o"]
            g, u = L["gate_up"].split([self.inter, self.inter])
            sd[p + "mlp.gate_proj.weight"], sd[p + "mlp.up_proj.weight"] = g, u
            sd[p + "mlp.down_proj.weight"] = L["down"]
            sd[p + "input_layernorm.weight"] = L["ln1"]
            sd[p + "post_attention_layernorm.weight"] = L["ln2"]
            if c.qkv_bias:
                qb, kb, vb = L["qkv_bias"].split([nq, nkv, nkv])
                sd[p + "self_attn.q_proj.bias"], sd[p + "self_attn.k_proj.bias"] = qb, kb
                sd[p + "self_attn.v_proj.bias"] = vb
            if c.qk_norm:
                sd[p + "self_attn.q_norm.weight"] = L["q_norm"]
                sd[p + "self_attn.k_norm.weight"] = L["k_norm"]
        sd["model.embed_tokens.weight"] = self.embed
        if not c.tie_embeddings:
            sd["lm_head.weight"] = self.lm_head
        sd["model.norm.weight"] = self.final_norm
        return {k: t.contiguous() for k, t in sd.items()}

    def _finish(self):
        from ..ops.reference import quantize_weight_fp8, rope_cache
        c = self.cfg
        if self.quant == "fp8":
            # per-output-channel e4m3fn weights (+ fp32 scales) replace the bf16 projections;
            # embedding, norms and the LM head stay bf16 (as vLLM's fp8 path)
            for L in self.layers:
                for name in self.PROJECTIONS:
                    if L[name].dtype != torch.float8_e4m3fn:
                        L[name], L[name + "_s"] = quantize_weight_fp8(L[name])
        self.cos_sin = rope_cache(min(c.max_position, 65536), self.hd, c.rope_theta, self.device)

    def weight_bytes(self) -> int:
        n = sum(t.numel() * t.element_size() for layer in self.layers for t in layer.values())
        n += self.embed.numel() * self.embed.element_size()
        if not self.cfg.tie_embeddings:
            n += self.lm_head.numel() * self.lm_head.element_size()
        return n

    # ------------------------------------------------------------- forward
    def forward(self, tokens: torch.Tensor, meta: AttnMeta, k_cache: torch.Tensor,
                v_cache: torch.Tensor) -> torch.Tensor:
        """Returns logits ``[len(logits_idx) or B, vocab]`` (full vocab, fp32 or bf16)."""
        if self.quant is None and self.tp.size == 1 and hasattr(self.ops, "linear_residual"):
            return self._forward_fused(tokens, meta, k_cache, v_cache)
        return self._forward_general(tokens, meta, k_cache, v_cache)

    @staticmethod
    def _last_layer_rows(meta, attn, residual):
        """Keep only the logits rows after the LAST layer's attention.

        Every row's o_proj / MLP / final norm is independent of the other rows, and past the
        last attention no later layer reads them: only the rows whose logits are sampled
        (``meta.logits_idx``, one per prompt that ends in this chunk) need the rest of the
        layer.  The K/V of every row is already in the cache (written in ``_attention``).
        In a packed prefill chunk that is the last layer's o / gate_up / down GEMMs on
        ~10-100 rows instead of up to 16384: ~1/40 of the chunk's GEMM work.  The residual
        stream of the previous layer is complete here (TP: reduced in this layer's input
        norm), so selecting it is exact; under TP every rank selects the same rows.
        """
        idx = meta.logits_idx
        return attn.index_select(0, idx), residual.index_select(0, idx)

    def _attention(self, li, L, qkv, meta, k_cache, v_cache):
        ops, c = self.ops, self.cfg
        q = ops.qk_norm_rope_kv_write(qkv, meta.positions, meta.slots, self.n_q, self.n_kv, self.hd,
                                      L.get("q_norm"), L.get("k_norm"), c.rms_eps, self.cos_sin,
                                      k_cache, v_cache, li, contiguous=not meta.decode)
        if meta.decode:
            lens = meta.seq_lens if meta.attn_seq_lens is None else meta.attn_seq_lens
            return ops.paged_attention_decode(q, k_cache, v_cache, li, meta.block_tables, lens,
                                              self.scale, meta.workspace, meta.cascade)
        return ops.paged_attention_prefill(q, k_cache, v_cache, li, meta.block_tables, meta.q_start,
                                           meta.seq_lens, self.scale, meta.max_q_len, meta.tiles,
                                           tile_rows=meta.tile_rows)

    def _forward_general(self, tokens, meta, k_cache, v_cache):
        """Tensor-parallel and / or fp8 forward, with the same fusions as the TP=1 bf16 path
        where the math allows them:

        * first layer: embedding gather + RMSNorm (+ fp8 quant) in one kernel;
        * TP (row-parallel o / down): the rank's partial output goes straight into the fused
          all-reduce + residual add + RMSNorm (xGMI kernel, RCCL + add_rmsnorm beyond it);
          under fp8 the row-wise quant follows on the normed rows;
        * TP=1 fp8: o / down add into the residual stream in the fp8 GEMM epilogue, then a
          plain RMSNorm + quant (no separate residual pass);
        * bf16 gate_up: SiLU * up fused into the GEMM epilogue (``linear_silu``) -- the
          column-parallel shard [gate_r; up_r] is local, so this holds under TP too;
        * fp8 gate_up: SiLU * up fused with the quant of the down projection's input;
        * the final norm and LM head run on the logits rows only (selected BEFORE the last
          all-reduce: the reduction is row-wise).
        """
        ops, c, tp = self.ops, self.cfg, self.tp
        fp8, tp1 = self.quant == "fp8", self.tp.size == 1
        eps = c.rms_eps
        residual = x = h = hq = hs = None
        last = len(self.layers) - 1
        for li, L in enumerate(self.layers):
            # ---- input norm (the previous layer's down projection is reduced here) ----
            if li == 0:
                if fp8:
                    hq, hs, residual = ops.embed_rmsnorm_fp8(tokens, self.embed, L["ln1"], eps)
                else:
                    h, residual = ops.embed_rmsnorm(tokens, self.embed, L["ln1"], eps)
            elif fp8 and tp1:
                hq, hs = ops.rmsnorm_fp8(residual, L["ln1"], eps)
            else:
                h, residual = tp.all_reduce_add_rmsnorm(x, residual, L["ln1"], eps, ops)
                if fp8:
                    hq, hs = ops.quant_fp8(h)
            qkv = (ops.linear_fp8(hq, hs, L["qkv"], L["qkv_s"], L.get("qkv_bias")) if fp8
                   else ops.linear(h, L["qkv"], L.get("qkv_bias")))
            attn = self._attention(li, L, qkv, meta, k_cache, v_cache)
            if li == last and meta.logits_idx is not None:  # see _last_layer_rows
                attn, residual = self._last_layer_rows(meta, attn, residual)
            # ---- o_proj, post-attention norm, MLP ----
            if fp8:
                aq, as_ = ops.quant_fp8(attn)
                if tp1:
                    ops.linear_fp8_residual(aq, as_, L["o"], L["o_s"], residual)
                    hq, hs = ops.rmsnorm_fp8(residual, L["ln2"], eps)
                else:
                    h, residual = tp.all_reduce_add_rmsnorm(ops.linear_fp8(aq, as_, L["o"], L["o_s"]), residual,
                                                            L["ln2"], eps, ops)
                    hq, hs = ops.quant_fp8(h)
                mq, ms = ops.silu_mul_fp8(ops.linear_fp8(hq, hs, L["gate_up"], L["gate_up_s"]))
                if tp1:
                    ops.linear_fp8_residual(mq, ms, L["down"], L["down_s"], residual)
                else:
                    x = ops.linear_fp8(mq, ms, L["down"], L["down_s"])  # partial: reduced at the next norm
            else:
                h, residual = tp.all_reduce_add_rmsnorm(ops.linear(attn, L["o"]), residual, L["ln2"], eps, ops)
                x = ops.linear(ops.linear_silu(h, L["gate_up"]), L["down"])  # partial: reduced at the next norm
        if tp1 and fp8:
            h = ops.rmsnorm(residual, self.final_norm, eps)
        else:
            h, _ = tp.all_reduce_add_rmsnorm(x, residual, self.final_norm, eps, ops)
        logits = ops.linear(h, self.lm_head)
        return tp.all_gather_last(logits)

    def _forward_fused(self, tokens, meta, k_cache, v_cache):
        """TP=1 bf16 forward with the GEMM epilogues fused (hand MFMA kernel where the
        GEMM plan picks it, ops/gemm_plan.py):

            o_proj   : residual <- residual + attn Wo^T       (+ plain RMSNorm after)
            gate_up  : h <- silu(x Wg^T) * (x Wu^T)           (K-ACT inside the GEMM)
            down     : residual <- residual + h Wd^T          (+ plain RMSNorm of the next layer)

        so the residual stream never takes a separate add pass and the [T, 2I]
        gate_up activation is never written to HBM.
        """
        ops, c = self.ops, self.cfg
        residual = None
        last = len(self.layers) - 1
        for li, L in enumerate(self.layers):
            if li == 0:  # embedding gather fused with the first input norm
                h, residual = ops.embed_rmsnorm(tokens, self.embed, L["ln1"], c.rms_eps)
            else:
                h = ops.rmsnorm(residual, L["ln1"], c.rms_eps)
            qkv = ops.linear(h, L["qkv"], L.get("qkv_bias"))
            attn = self._attention(li, L, qkv, meta, k_cache, v_cache)
            if li == last and meta.logits_idx is not None:  # see _last_layer_rows
                attn, residual = self._last_layer_rows(meta, attn, residual)
            residual = ops.linear_residual(attn, L["o"], residual)
            h = ops.rmsnorm(residual, L["ln2"], c.rms_eps)
            act = ops.linear_silu(h, L["gate_up"])
            residual = ops.linear_residual(act, L["down"], residual)
        h = ops.rmsnorm(residual, self.final_norm, c.rms_eps)
        return ops.linear(h, self.lm_head)
