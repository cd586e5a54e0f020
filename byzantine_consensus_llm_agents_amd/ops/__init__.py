"""Op dispatch: ``get_ops("hip")`` -> HIP/CDNA4 kernels, ``get_ops("torch")`` -> references.

Both namespaces expose the same functions (see ``reference.py`` for the
semantics).  The HIP namespace raises at import when ``libbcg_kernels.so``
is missing instead of silently falling back.
"""

from types import SimpleNamespace

import torch

from . import reference as _ref


def _torch_ops() -> SimpleNamespace:
    def decode(q, k_cache, v_cache, layer, block_tables, seq_lens, scale, workspace=None, cascade=None):
        # the shared-prefix cascade changes how the kernel walks the KV, not the result
        B = q.shape[0]
        q_start = torch.arange(B + 1, dtype=torch.int32, device=q.device)
        return _ref.paged_attention(q, k_cache, v_cache, layer, block_tables, q_start, seq_lens, scale)

    def prefill(q, k_cache, v_cache, layer, block_tables, q_start, seq_lens, scale, max_q_len=None, tiles=None,
                tile_rows=64):
        return _ref.paged_attention(q, k_cache, v_cache, layer, block_tables, q_start, seq_lens, scale)

    return SimpleNamespace(
        name="torch",
        linear=torch.nn.functional.linear,
        rmsnorm=_ref.rmsnorm,
        add_rmsnorm=_ref.add_rmsnorm,
        embed_rmsnorm=_ref.embed_rmsnorm,
        qk_norm_rope_kv_write=_ref.qk_norm_rope_kv_write,
        paged_attention_decode=decode,
        paged_attention_prefill=prefill,
        prefill_tile_rows=lambda hd, kv_fp8=False, max_blocks=0: 64,
        silu_mul=_ref.silu_mul,
        linear_silu=_ref.linear_silu,
        linear_residual=_ref.linear_residual,
        sample_step=_ref.sample_step,
        quant_fp8=_ref.quant_fp8,
        add_rmsnorm_fp8=_ref.add_rmsnorm_fp8,
        silu_mul_fp8=_ref.silu_mul_fp8,
        linear_fp8=_ref.linear_fp8,
        rmsnorm_fp8=_ref.rmsnorm_fp8,
        embed_rmsnorm_fp8=_ref.embed_rmsnorm_fp8,
        linear_fp8_residual=_ref.linear_fp8_residual,
    )


_CACHE = {}


def get_ops(backend: str) -> SimpleNamespace:
    if backend not in _CACHE:
        if backend == "torch":
            _CACHE[backend] = _torch_ops()
        elif backend == "hip":
            from .hip import hip_ops
            _CACHE[backend] = hip_ops()
        else:
            raise ValueError(f"unknown ops backend {backend!r}")
    return _CACHE[backend]
