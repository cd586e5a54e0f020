"""ctypes bindings of ``libbcg_kernels.so`` (csrc/kernels, gfx950).

Every wrapper validates dtypes, contiguity and shapes on the host before it
launches (a kernel that indexes out of bounds can take down every GPU of the
node), then launches on the current HIP stream -- so the calls are captured
by ``torch.cuda.graph`` like any PyTorch op.  A missing library raises: on a
GPU box the engine never silently falls back to the PyTorch references.
"""

import ctypes
import os
from types import SimpleNamespace

import torch

from ..utils.build import kernel_sources, kernels_source_hash, kernels_target

_LIB = None
# Rows per prefill attention tile unless BCG_PREFILL_TILE_ROWS says otherwise (prefill_tile_rows)
PREFILL_TILE_ROWS = 128
PREFILL32_MAX_BLOCKS = 1024  # csrc/kernels/attention.hip: the 32x32 kernel's LDS block-id table

c_int, c_float, c_void_p, c_uint32, c_int64 = ctypes.c_int, ctypes.c_float, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int64


class StaleLibraryError(RuntimeError):
    pass


def library_stamp(lib: ctypes.CDLL) -> str:
    fn = getattr(lib, "bcg_source_hash", None)
    if fn is None:
        return None
    fn.argtypes, fn.restype = [], ctypes.c_char_p
    return fn().decode()


def check_source_stamp(lib: ctypes.CDLL, path: str):
    """Refuse a library built from other sources than the tree's csrc/kernels.

    ``utils/build.py`` stamps the library with a hash of every kernel source.
    A deployment without sources (no csrc/kernels) has nothing to compare with
    and is accepted."""
    if not kernel_sources()[0]:
        return
    want, got = kernels_source_hash(), library_stamp(lib)
    if got != want:
        raise StaleLibraryError(
            f"{path} was built from other sources (stamp {got!r}, csrc/kernels {want!r}); rebuild with "
            "`python -m byzantine_consensus_llm_agents_amd.utils.build --force`")


def load_library(path: str = None) -> ctypes.CDLL:
    global _LIB
    if _LIB is not None:
        return _LIB
    path = path or os.environ.get("BCG_KERNELS_LIB") or kernels_target()  # override: variant builds (tools)
    if not os.path.exists(path):
        raise RuntimeError(f"HIP kernel library not found at {path}; run `python -m "
                           "byzantine_consensus_llm_agents_amd.utils.build` (hipcc --offload-arch=gfx950)")
    lib = ctypes.CDLL(path)
    check_source_stamp(lib, path)
    sig = {
        "bcg_add_rmsnorm": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_int, c_void_p],
        "bcg_silu_mul": [c_void_p, c_void_p, c_int64, c_int, c_void_p],
        "bcg_embed_rmsnorm": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_void_p],
        "bcg_qk_norm_rope_kv_write": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                      c_float, c_int, c_int, c_void_p],
        "bcg_paged_attention_decode": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int,
                                       c_void_p, c_int, c_int, c_int, c_int, c_float, c_void_p, c_int,
                                       c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                                       c_int, c_void_p, c_void_p, c_int, c_int, c_void_p],
        "bcg_paged_attention_prefill": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int,
                                        c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float,
                                        c_void_p, c_int, c_int, c_void_p],
        "bcg_paged_attention_prefill32": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int,
                                          c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float,
                                          c_void_p, c_int, c_int, c_void_p],
        "bcg_decode_split_tokens": [c_int, c_int, c_int],
        "bcg_decode_max_splits": [c_int, c_int],
        "bcg_decode_max_context": [c_int],
        "bcg_quant_fp8": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p],
        "bcg_add_rmsnorm_fp8": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_int,
                                c_void_p],
        "bcg_silu_mul_fp8": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p],
        "bcg_embed_rmsnorm_fp8": [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float,
                                  c_void_p],
        "bcg_gemm_nt": [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                        c_int, c_int, c_int, c_int, c_int, c_void_p],
        "bcg_gemm_nt_fp8": [c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                            c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p],
        "bcg_gemm_tile": [c_int, ctypes.POINTER(c_int), ctypes.POINTER(c_int)],
        "bcg_gemm_num_cfgs": [],
        "bcg_guided_sample": [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                              c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p,
                              c_uint32, c_int, c_int, c_int, c_int, c_void_p],
    }
    for name, argtypes in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = c_int
    _LIB = lib
    return lib


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _p(t: torch.Tensor):
    return ctypes.c_void_p(t.data_ptr())


def _check(rc: int, name: str):
    if rc != 0:
        raise RuntimeError(f"{name} launch failed (rc={rc})")


def _req(cond: bool, msg: str):
    if not cond:
        raise ValueError(msg)


def _kv_fp8(k_cache: torch.Tensor, v_cache: torch.Tensor) -> int:
    """1 for an fp8 (e4m3fn) KV cache, 0 for bf16; anything else is refused before launch."""
    _req(k_cache.dtype == v_cache.dtype and k_cache.dtype in (torch.bfloat16, torch.float8_e4m3fn)
         and k_cache.is_contiguous() and v_cache.is_contiguous(), "KV cache: contiguous bf16 or float8_e4m3fn")
    return int(k_cache.dtype == torch.float8_e4m3fn)


def hip_ops() -> SimpleNamespace:
    lib = load_library()

    def add_rmsnorm(x, residual, w, eps):
        _req(x.dtype == torch.bfloat16 and x.is_contiguous() and x.dim() == 2, "add_rmsnorm: x bf16 [T,H]")
        T, H = x.shape
        _req(w.shape == (H,) and w.dtype == torch.bfloat16, "add_rmsnorm: weight [H] bf16")
        has_res = residual is not None
        if not has_res:
            residual = torch.empty_like(x)
        else:
            _req(residual.shape == x.shape and residual.is_contiguous(), "add_rmsnorm: residual shape")
        out = torch.empty_like(x)
        _check(lib.bcg_add_rmsnorm(_p(x), _p(residual), _p(w), _p(out), T, H, eps, int(has_res), _stream()),
               "add_rmsnorm")
        return out, residual

    def embed_rmsnorm(tokens, table, w, eps):
        """(rmsnorm(table[tokens]) * w, table[tokens]) in one pass over the gathered rows."""
        _req(tokens.dtype == torch.int32 and tokens.is_contiguous() and tokens.dim() == 1, "tokens int32 [T]")
        _req(table.dtype == torch.bfloat16 and table.is_contiguous() and table.dim() == 2, "table bf16 [V,H]")
        T, H = tokens.numel(), table.shape[1]
        _req(w.shape == (H,) and w.dtype == torch.bfloat16, "embed_rmsnorm: weight [H] bf16")
        residual = torch.empty(T, H, dtype=table.dtype, device=table.device)
        out = torch.empty_like(residual)
        _check(lib.bcg_embed_rmsnorm(_p(tokens), _p(table), _p(w), _p(residual), _p(out), T, H, eps, _stream()),
               "embed_rmsnorm")
        return out, residual

    def rmsnorm(x, w, eps):
        """Plain RMSNorm (mode 2: the residual stream is not touched)."""
        _req(x.dtype == torch.bfloat16 and x.is_contiguous() and x.dim() == 2, "rmsnorm: x bf16 [T,H]")
        T, H = x.shape
        _req(w.shape == (H,) and w.dtype == torch.bfloat16, "rmsnorm: weight [H] bf16")
        out = torch.empty_like(x)
        _check(lib.bcg_add_rmsnorm(_p(x), None, _p(w), _p(out), T, H, eps, 2, _stream()), "rmsnorm")
        return out

    def silu_mul(gu):
        _req(gu.dtype == torch.bfloat16 and gu.is_contiguous() and gu.dim() == 2, "silu_mul: bf16 [T,2I]")
        T, I2 = gu.shape
        out = torch.empty(T, I2 // 2, dtype=gu.dtype, device=gu.device)
        _check(lib.bcg_silu_mul(_p(gu), _p(out), T, I2 // 2, _stream()), "silu_mul")
        return out

    def qk_norm_rope_kv_write(qkv, positions, slots, n_q, n_kv, head_dim, q_norm, k_norm, eps, cos_sin,
                              k_cache, v_cache, layer, contiguous=True):
        """contiguous: the tokens come in runs of consecutive slots (prefill chunks), so V can be
        written a whole KV block at a time; False for decode batches (one token per sequence)."""
        T = qkv.shape[0]
        _req(qkv.is_contiguous() and qkv.shape[1] == (n_q + 2 * n_kv) * head_dim, "qkv shape")
        _req(positions.dtype == torch.int32 and slots.dtype == torch.int32 and positions.numel() == T
             and slots.numel() == T, "positions/slots int32 [T]")
        _req(cos_sin.dtype == torch.float32 and cos_sin.shape[1] == head_dim, "cos_sin table")
        L, NB, nkv_c, BS, hd = k_cache.shape
        _req(nkv_c == n_kv and hd == head_dim and v_cache.shape == (L, NB, n_kv, hd, BS), "kv cache layout")
        q = torch.empty(T, n_q, head_dim, dtype=qkv.dtype, device=qkv.device)
        _check(lib.bcg_qk_norm_rope_kv_write(
            _p(qkv), _p(positions), _p(slots), _p(q), _p(q_norm) if q_norm is not None else None,
            _p(k_norm) if k_norm is not None else None, _p(cos_sin), _p(k_cache), _p(v_cache), layer, T,
            n_q, n_kv, head_dim, NB, BS, eps, _kv_fp8(k_cache, v_cache), int(bool(contiguous)), _stream()),
            "qk_norm_rope_kv_write")
        return q

    def decode_workspace_numel(B, n_q, hd, max_blocks, block_size=16, cascade=True):
        """fp32 split partials (o, m, l) of the flash-decoding split-K (+ the shared-prefix
        pass's slots when `cascade`)."""
        max_splits = lib.bcg_decode_max_splits(max_blocks * block_size, int(cascade))
        return B * n_q * max_splits * (hd + 2)

    def paged_attention_decode(q, k_cache, v_cache, layer, block_tables, seq_lens, scale, workspace=None,
                               cascade=None):
        """`workspace`: optional fp32 split-K scratch of >= decode_workspace_numel(...) elements,
        shared by every decode graph (it is dead between launches) instead of one per graph.
        `cascade`: optional shared-prefix tables (``engine/cascade.py`` ``CascadeTables``):
        rows whose leading KV blocks are shared read them once per group."""
        B, n_q, hd = q.shape
        L, NB, n_kv, BS, _ = k_cache.shape
        _req(q.is_contiguous() and block_tables.dtype == torch.int32 and block_tables.is_contiguous()
             and block_tables.shape[0] == B and seq_lens.numel() == B, "decode attention inputs")
        max_blocks = block_tables.shape[1]
        _req(B <= 2048, "decode attention: at most 2048 rows")
        split = lib.bcg_decode_split_tokens(B, n_kv, max_blocks * BS)
        max_splits = lib.bcg_decode_max_splits(max_blocks * BS, int(cascade is not None))
        need = B * n_q * max_splits * (hd + 2)
        if workspace is None:
            ws = torch.empty(need, dtype=torch.float32, device=q.device)
        else:
            _req(workspace.dtype == torch.float32 and workspace.is_contiguous() and workspace.numel() >= need,
                 "decode attention workspace too small")
            ws = workspace
        cas = [None, None, None, 0, None, 0, None, None, 0, 32]
        if cascade is not None:
            c = cascade
            i32 = torch.int32
            for t in (c.kv_begin, c.split_base, c.grp_rows, c.grp_desc, c.items, c.n_items):
                _req(t.dtype == i32 and t.is_contiguous() and t.device == q.device, "cascade tables: int32 on device")
            _req(c.kv_begin.numel() >= B and c.split_base.numel() >= B, "cascade tables: one entry per row")
            _req(c.grp_desc.dim() == 2 and c.grp_desc.shape[1] == 4 and c.items.dim() == 2 and c.items.shape[1] == 4
                 and c.n_items.numel() >= 1, "cascade tables: grp_desc [G, 4], items [I, 4], n_items [1]")
            cas = [_p(c.kv_begin), _p(c.split_base), _p(c.grp_rows), c.grp_rows.numel(), _p(c.grp_desc),
                   c.grp_desc.shape[0], _p(c.items), _p(c.n_items), c.items.shape[0], c.split_tokens]
        out = torch.empty(B, n_q * hd, dtype=q.dtype, device=q.device)
        _check(lib.bcg_paged_attention_decode(
            _p(q), _p(k_cache), _p(v_cache), layer, NB, n_kv, _p(block_tables), max_blocks, _p(seq_lens),
            B, n_q, hd, BS, scale, _p(ws), max_splits, split, _p(out), _kv_fp8(k_cache, v_cache), *cas,
            _stream()), "paged_attention_decode")
        return out

    def paged_attention_prefill(q, k_cache, v_cache, layer, block_tables, q_start, seq_lens, scale,
                                max_q_len=None, tiles=None, tile_rows=64):
        """tiles: [n_tiles, 3] int32 {sequence, first row, end row} of at most `tile_rows` rows.
        64-row tiles run the 16x16 register kernel; 128 / 256-row tiles the LDS-staged 32x32
        kernel (bf16 KV cache, head dim 128: `prefill_tile_rows` says which the engine builds)."""
        T, n_q, hd = q.shape
        L, NB, n_kv, BS, _ = k_cache.shape
        _req(tiles is not None and tiles.dtype == torch.int32 and tiles.dim() == 2 and tiles.shape[1] == 3,
             "prefill attention needs the [n_tiles,3] int32 tile table")
        _req(q.is_contiguous() and block_tables.dtype == torch.int32 and q_start.dtype == torch.int32
             and seq_lens.dtype == torch.int32, "prefill attention inputs")
        out = torch.empty(T, n_q * hd, dtype=q.dtype, device=q.device)
        if tile_rows != 64:
            _req(tile_rows in (128, 256) and hd == 128 and not _kv_fp8(k_cache, v_cache),
                 "32x32 prefill attention: 128 / 256-row tiles, head dim 128, bf16 KV cache")
            _check(lib.bcg_paged_attention_prefill32(
                _p(q), _p(k_cache), _p(v_cache), layer, NB, n_kv, _p(block_tables), block_tables.shape[1],
                _p(q_start), _p(seq_lens), _p(tiles), tiles.shape[0], n_q, hd, BS, scale, _p(out),
                tile_rows, 0, _stream()), "paged_attention_prefill32")
            return out
        _check(lib.bcg_paged_attention_prefill(
            _p(q), _p(k_cache), _p(v_cache), layer, NB, n_kv, _p(block_tables), block_tables.shape[1],
            _p(q_start), _p(seq_lens), _p(tiles), tiles.shape[0], n_q, hd, BS, scale, _p(out),
            4, _kv_fp8(k_cache, v_cache), _stream()), "paged_attention_prefill")
        return out

    def prefill_tile_rows(hd, kv_fp8=False, max_blocks=0):
        """Rows per prefill attention tile for this geometry (the tile table the caller builds):
        128 / 256 select the LDS-staged 32x32 kernel (head dim 128, bf16 KV, block tables of at
        most 1024 entries -- 16k tokens -- which it stages in LDS), 64 the 16x16 one.
        BCG_PREFILL_TILE_ROWS overrides the default."""
        rows = int(os.environ.get("BCG_PREFILL_TILE_ROWS", PREFILL_TILE_ROWS))
        ok = rows in (128, 256) and hd == 128 and not kv_fp8 and max_blocks <= PREFILL32_MAX_BLOCKS
        return rows if ok else 64

    # Per-call GEMM dispatch log (which projection shapes reach a hand kernel, also
    # inside TP worker processes that no profiler sees): (M, N, K, epi, dtype) -> choice -> calls.
    # Off unless enabled (BCG_GEMM_LOG=1 or dispatch_log.enable()); graph-captured calls are
    # logged once, at capture (the replays run the same kernels).
    dispatch_log = SimpleNamespace(enabled=os.environ.get("BCG_GEMM_LOG") == "1", calls={})

    def _log(M, N, K, epi, choice, dtype="bf16"):
        if dispatch_log.enabled:
            key = (M, N, K, epi, dtype, "lib" if choice is None else f"{choice[0]}x{choice[1]}")
            dispatch_log.calls[key] = dispatch_log.calls.get(key, 0) + 1

    def linear(x, w, bias=None, _epi_log=0):
        """y = x W^T (+b): hand MFMA GEMM where the plan says it beats hipBLASLt, hipBLASLt otherwise."""
        M, K = x.shape
        N = w.shape[0]
        cfg = None
        if x.is_contiguous() and x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16:
            cfg = plan.choose(M, N, K, 0)
        _log(M, N, K, _epi_log, cfg)
        if cfg is not None:
            return gemm_nt(x, w, cfg, 0, bias=bias)
        return torch.nn.functional.linear(x, w, bias)

    from .gemm_plan import PP_CFG, W4_CFG, GemmPlan
    plan = GemmPlan(lib)

    # Split-K arrival counters (one int per output tile; the last-arriving workgroup of a
    # tile resets its counter, so a buffer stays zero between launches).  Kernels that may
    # run CONCURRENTLY need disjoint buffers: one per device for the engine's main stream --
    # shared by eager launches and every captured decode graph, which replay on that stream
    # one after another -- and one per registered side stream.  Buffers are allocated eagerly
    # by `prepare_device` / `register_stream`, never inside a graph capture: a zero-fill captured into one bucket's graph would leave the
    # buffer uninitialised for every other graph.
    counters = {}       # device index -> int32 [65536]
    side_counters = {}  # (device index, stream handle) -> int32 [65536]

    def _new_counters(dev):
        _req(not torch.cuda.is_current_stream_capturing(),
             "split-K counters must be allocated outside graph capture (ops.prepare_device)")
        return torch.zeros(1 << 16, dtype=torch.int32, device=dev)

    sk_ws = {}  # device index -> fp32 [2 x CUs x 65536]: stream-K parts (W4, split_k == 0)

    def prepare_device(dev):
        dev = torch.device(dev)
        if dev.index is None:
            dev = torch.device("cuda", torch.cuda.current_device())
        if dev.index not in counters:
            counters[dev.index] = _new_counters(dev)
        if dev.index not in sk_ws:  # (128 MiB; allocated outside any graph capture)
            with torch.cuda.device(dev):
                sk_ws[dev.index] = torch.empty(lib.bcg_gemm_w4_sk_ws_floats(), dtype=torch.float32, device=dev)

    def _sk_workspace(dev):
        dev = torch.device("cuda", dev.index if dev.index is not None else torch.cuda.current_device())
        if dev.index not in sk_ws:
            prepare_device(dev)  # raises under capture (the counters' check)
        return sk_ws[dev.index]

    def register_stream(stream):
        """Give `stream` its own split-K counters (its GEMMs may overlap the main stream's)."""
        key = (stream.device.index, stream.cuda_stream)
        if key not in side_counters:
            side_counters[key] = _new_counters(stream.device)

    def _counters(dev):
        dev = torch.device("cuda", dev.index if dev.index is not None else torch.cuda.current_device())
        side = side_counters.get((dev.index, torch.cuda.current_stream(dev).cuda_stream))
        if side is not None:
            return side
        if dev.index not in counters:
            prepare_device(dev)  # raises under capture
        return counters[dev.index]

    def gemm_nt(x, w, cfg, epi=0, bias=None, residual=None, out=None, split_k=1):
        """Hand MFMA GEMM (csrc/kernels/gemm.hip): x [M,K] @ w[N,K]^T with epilogue `epi`
        (0 store(+bias), 1 silu(gate)*up -> [M, N/2], 2 residual + acc); `split_k` K-slices
        reduced in the kernel by the last-arriving workgroup of each tile."""
        if isinstance(cfg, (tuple, list)):
            cfg, split_k = cfg
        M, K = x.shape
        N = w.shape[0]
        _req(x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and x.is_contiguous() and w.is_contiguous()
             and w.shape[1] == K, "gemm_nt: contiguous bf16 x [M,K], w [N,K]")
        _req(plan.supported(cfg, M, N, K, epi, split_k),
             f"gemm_nt: shape {M}x{N}x{K} epi {epi} split {split_k} unsupported by tile {cfg}")
        width = N // 2 if epi == 1 else N
        if out is None:
            out = torch.empty(M, width, dtype=x.dtype, device=x.device)
        _req(out.shape == (M, width) and out.is_contiguous() and out.dtype == torch.bfloat16, "gemm_nt: out")
        if bias is not None:
            _req(bias.shape == (N,) and bias.dtype == torch.bfloat16 and bias.is_contiguous(), "gemm_nt: bias")
        if epi == 2:
            _req(residual is not None and residual.shape == (M, N) and residual.is_contiguous()
                 and residual.dtype == torch.bfloat16, "gemm_nt: residual [M,N] bf16")
        ws = cnt = None
        if split_k == 0:  # W4 stream-K: the device's persistent part buffer + the counters
            ws, cnt = _sk_workspace(x.device), _counters(x.device)
        elif split_k > 1:
            bm, bn = plan.tiles[cfg]
            tiles = (M + bm - 1) // bm * ((N + bn - 1) // bn)
            _req(tiles <= (1 << 16), "gemm_nt: too many output tiles for split-K")
            ws = torch.empty(tiles * split_k * bm * bn, dtype=torch.float32, device=x.device)
            cnt = _counters(x.device)
        _check(lib.bcg_gemm_nt(cfg, epi, _p(x), _p(w), _p(bias) if bias is not None else None,
                               _p(residual) if residual is not None else None, _p(out),
                               _p(ws) if ws is not None else None, _p(cnt) if cnt is not None else None,
                               M, N, K, N // 2, split_k, _stream()), "gemm_nt")
        return out

    def linear_silu(x, w):
        """silu(x Wg^T) * (x Wu^T), W = [gate; up] -- K-ACT fused into the gate_up GEMM."""
        M, K = x.shape
        cfg = plan.choose(M, w.shape[0], K, 1) if x.is_contiguous() and x.dtype == torch.bfloat16 else None
        if cfg is None:
            return silu_mul(linear(x, w, _epi_log=1))
        _log(M, w.shape[0], K, 1, cfg)
        return gemm_nt(x, w, cfg, 1)

    residual_addmm = os.environ.get("BCG_RESIDUAL_ADDMM", "1") == "1"

    def linear_residual(x, w, residual):
        """residual <- residual + x W^T (in place; the o/down projection fused with the
        residual-stream update of the next add+RMSNorm).  Returns `residual`."""
        M, K = x.shape
        cfg = plan.choose(M, w.shape[0], K, 2) if x.is_contiguous() and x.dtype == torch.bfloat16 else None
        _log(M, w.shape[0], K, 2, cfg)
        if cfg is None:
            if (residual_addmm and residual.is_contiguous() and residual.dtype == x.dtype == w.dtype
                    and residual.shape == (M, w.shape[0])):
                # hipBLASLt with beta = 1: the residual add rides in the GEMM epilogue (one read
                # of the residual, no separate elementwise pass over three [M, H] tensors)
                return residual.addmm_(x, w.t())
            residual.add_(torch.nn.functional.linear(x, w))
            return residual
        return gemm_nt(x, w, cfg, 2, residual=residual, out=residual)

    def sample_step(logits, fsm_next, fsm_dist, fsm_base, fsm_state, gen_count, max_new, temperature,
                    row_keys, done, seq_lens, out_tokens, next_tokens, seed, budget_aware, n_text_tokens,
                    eos_id, eos_id2):
        B, V = logits.shape
        _req(logits.dtype == torch.bfloat16 and logits.is_contiguous(), "logits bf16 [B,V]")
        _req(fsm_next.dtype == torch.int16 and fsm_next.shape[1] == V and fsm_dist.dtype == torch.int16,
             "fsm tables int16 [rows,V]")
        for t in (fsm_base, fsm_state, gen_count, max_new, row_keys, done, seq_lens, next_tokens):
            _req(t.dtype == torch.int32 and t.numel() == B and t.is_contiguous(), "per-row int32 state")
        _req(temperature.dtype == torch.float32 and out_tokens.dtype == torch.int32
             and out_tokens.shape[0] == B, "temperature/out_tokens")
        _check(lib.bcg_guided_sample(
            _p(logits), B, V, _p(fsm_next), _p(fsm_dist), _p(fsm_base), _p(fsm_state), _p(gen_count),
            _p(max_new), _p(temperature), _p(row_keys), _p(done), _p(seq_lens), _p(out_tokens),
            out_tokens.shape[1], _p(next_tokens), seed & 0xFFFFFFFF, int(bool(budget_aware)), n_text_tokens,
            eos_id, eos_id2, _stream()), "guided_sample")

    f8 = torch.float8_e4m3fn

    def quant_fp8(x):
        _req(x.dtype == torch.bfloat16 and x.is_contiguous() and x.dim() == 2 and x.shape[1] % 8 == 0,
             "quant_fp8: bf16 [T,K], K % 8 == 0")
        T, K = x.shape
        q = torch.empty(T, K, dtype=f8, device=x.device)
        s = torch.empty(T, dtype=torch.float32, device=x.device)
        _check(lib.bcg_quant_fp8(_p(x), _p(q), _p(s), T, K, _stream()), "quant_fp8")
        return q, s

    def add_rmsnorm_fp8(x, residual, w, eps):
        _req(x.dtype == torch.bfloat16 and x.is_contiguous() and x.dim() == 2, "add_rmsnorm_fp8: x bf16 [T,H]")
        T, H = x.shape
        _req(w.shape == (H,) and w.dtype == torch.bfloat16, "add_rmsnorm_fp8: weight [H] bf16")
        has_res = residual is not None
        if not has_res:
            residual = torch.empty_like(x)
        else:
            _req(residual.shape == x.shape and residual.is_contiguous(), "add_rmsnorm_fp8: residual shape")
        q = torch.empty(T, H, dtype=f8, device=x.device)
        s = torch.empty(T, dtype=torch.float32, device=x.device)
        _check(lib.bcg_add_rmsnorm_fp8(_p(x), _p(residual), _p(w), _p(q), _p(s), T, H, eps, int(has_res),
                                       _stream()), "add_rmsnorm_fp8")
        return q, s, residual

    def rmsnorm_fp8(x, w, eps):
        """Plain RMSNorm + row-wise fp8 quant (the residual stream was updated by the GEMM epilogue)."""
        _req(x.dtype == torch.bfloat16 and x.is_contiguous() and x.dim() == 2, "rmsnorm_fp8: x bf16 [T,H]")
        T, H = x.shape
        _req(w.shape == (H,) and w.dtype == torch.bfloat16, "rmsnorm_fp8: weight [H] bf16")
        q = torch.empty(T, H, dtype=f8, device=x.device)
        s = torch.empty(T, dtype=torch.float32, device=x.device)
        _check(lib.bcg_add_rmsnorm_fp8(_p(x), None, _p(w), _p(q), _p(s), T, H, eps, 2, _stream()), "rmsnorm_fp8")
        return q, s

    def embed_rmsnorm_fp8(tokens, table, w, eps):
        """(fp8(rmsnorm(table[tokens]) * w), row scales, table[tokens]) in one pass."""
        _req(tokens.dtype == torch.int32 and tokens.is_contiguous() and tokens.dim() == 1, "tokens int32 [T]")
        _req(table.dtype == torch.bfloat16 and table.is_contiguous() and table.dim() == 2, "table bf16 [V,H]")
        T, H = tokens.numel(), table.shape[1]
        _req(w.shape == (H,) and w.dtype == torch.bfloat16, "embed_rmsnorm_fp8: weight [H] bf16")
        residual = torch.empty(T, H, dtype=table.dtype, device=table.device)
        q = torch.empty(T, H, dtype=f8, device=table.device)
        s = torch.empty(T, dtype=torch.float32, device=table.device)
        _check(lib.bcg_embed_rmsnorm_fp8(_p(tokens), _p(table), _p(w), _p(residual), _p(q), _p(s), T, H, eps,
                                         _stream()), "embed_rmsnorm_fp8")
        return q, s, residual

    def silu_mul_fp8(gu):
        _req(gu.dtype == torch.bfloat16 and gu.is_contiguous() and gu.dim() == 2 and gu.shape[1] % 16 == 0,
             "silu_mul_fp8: bf16 [T,2I]")
        T, I2 = gu.shape
        q = torch.empty(T, I2 // 2, dtype=f8, device=gu.device)
        s = torch.empty(T, dtype=torch.float32, device=gu.device)
        _check(lib.bcg_silu_mul_fp8(_p(gu), _p(q), _p(s), T, I2 // 2, _stream()), "silu_mul_fp8")
        return q, s

    def gemm_nt_fp8(xq, xs, wq, ws, cfg, epi=0, bias=None, residual=None, out=None, split_k=1):
        """Hand fp8 MFMA GEMM (csrc/kernels/gemm.hip, F8): xs[m] * ws[n] * (xq . wq^T)
        (+ bias) (+ residual when epi == 2), e4m3fn operands, bf16 out."""
        if isinstance(cfg, (tuple, list)):
            cfg, split_k = cfg
        M, K = xq.shape
        N = wq.shape[0]
        _req(xq.dtype == f8 and wq.dtype == f8 and xq.is_contiguous() and wq.is_contiguous() and wq.shape[1] == K,
             "gemm_nt_fp8: contiguous e4m3fn xq [M,K], wq [N,K]")
        _req(xs.dtype == torch.float32 and xs.numel() == M and xs.is_contiguous() and ws.dtype == torch.float32
             and ws.numel() == N and ws.is_contiguous(), "gemm_nt_fp8: fp32 scales xs [M], ws [N]")
        bm, bn = plan.tiles[cfg]
        pp = cfg == PP_CFG  # 256 x 256 ping-pong kernel: N only a multiple of 16, 32-bit buffer offsets
        w4 = cfg == W4_CFG  # four-wave 256 x 256 kernel: N a multiple of 16, offsets below 2 GiB
        _req(0 <= cfg <= W4_CFG and K % 128 == 0 and N % (16 if pp or w4 else bn) == 0 and 1 <= split_k <= K // 128
             and epi in (0, 2) and (not pp or (M * K < 1 << 32 and N * K < 1 << 32))
             and (not w4 or ((M + 256) * K < 1 << 31 and (N + 256) * K < 1 << 31))
             and (not (pp or w4) or 2 * (M + 256) * N < 1 << 31),
             f"gemm_nt_fp8: shape {M}x{N}x{K} epi {epi} split {split_k} unsupported by tile {cfg}")
        if out is None:
            out = torch.empty(M, N, dtype=torch.bfloat16, device=xq.device)
        _req(out.shape == (M, N) and out.is_contiguous() and out.dtype == torch.bfloat16, "gemm_nt_fp8: out")
        if bias is not None:
            _req(bias.shape == (N,) and bias.dtype == torch.bfloat16 and bias.is_contiguous(), "gemm_nt_fp8: bias")
        if epi == 2:
            _req(residual is not None and residual.shape == (M, N) and residual.is_contiguous()
                 and residual.dtype == torch.bfloat16, "gemm_nt_fp8: residual [M,N] bf16")
        wsp = cnt = None
        if split_k > 1:
            tiles = (M + bm - 1) // bm * ((N + bn - 1) // bn)
            _req(tiles <= (1 << 16), "gemm_nt_fp8: too many output tiles for split-K")
            wsp = torch.empty(tiles * split_k * bm * bn, dtype=torch.float32, device=xq.device)
            cnt = _counters(xq.device)
        _check(lib.bcg_gemm_nt_fp8(cfg, epi, _p(xq), _p(wq), _p(xs), _p(ws), _p(bias) if bias is not None else None,
                                   _p(residual) if residual is not None else None, _p(out),
                                   _p(wsp) if wsp is not None else None, _p(cnt) if cnt is not None else None,
                                   M, N, K, split_k, _stream()), "gemm_nt_fp8")
        return out

    from .gemm_plan import Fp8Plan
    fp8_plan = Fp8Plan(plan.tiles)
    fp8_cfg = fp8_plan.choose

    def linear_fp8(xq, xs, wq, ws, bias=None, out_dtype=torch.bfloat16):
        """fp8 projection with row-wise activation and per-channel weight scales: the hand
        fp8 MFMA kernel for decode-sized M, hipBLASLt (torch._scaled_mm) otherwise."""
        _req(xq.dtype == f8 and wq.dtype == f8 and xq.shape[1] == wq.shape[1], "linear_fp8 operands")
        cfg = None
        if out_dtype == torch.bfloat16 and xq.is_contiguous() and wq.is_contiguous():
            cfg = fp8_cfg(xq.shape[0], wq.shape[0], xq.shape[1])
        _log(xq.shape[0], wq.shape[0], xq.shape[1], 0, cfg, "fp8")
        if cfg is not None:
            return gemm_nt_fp8(xq, xs.contiguous(), wq, ws.contiguous(), cfg, 0, bias=bias)
        return torch._scaled_mm(xq, wq.t(), scale_a=xs.view(-1, 1), scale_b=ws.view(1, -1), bias=bias,
                                out_dtype=out_dtype)

    def linear_fp8_residual(xq, xs, wq, ws, residual):
        """residual <- residual + dequant(xq . wq^T) in place: the o/down projection's residual
        update in the hand fp8 kernel's epilogue (hipBLASLt + a separate add otherwise)."""
        _req(residual.dtype == torch.bfloat16 and residual.is_contiguous()
             and residual.shape == (xq.shape[0], wq.shape[0]), "linear_fp8_residual: residual [M,N] bf16")
        if xq.is_contiguous() and wq.is_contiguous():
            cfg = fp8_cfg(xq.shape[0], wq.shape[0], xq.shape[1])
            if cfg is not None:
                return gemm_nt_fp8(xq, xs.contiguous(), wq, ws.contiguous(), cfg, 2, residual=residual,
                                   out=residual)
        return residual.add_(linear_fp8(xq, xs, wq, ws))

    return SimpleNamespace(name="hip", rmsnorm_fp8=rmsnorm_fp8, embed_rmsnorm_fp8=embed_rmsnorm_fp8,
                           linear_fp8_residual=linear_fp8_residual, linear=linear, linear_silu=linear_silu, linear_residual=linear_residual,
                           gemm_nt=gemm_nt, gemm_plan=plan, prepare_device=prepare_device,
                           register_stream=register_stream, quant_fp8=quant_fp8, add_rmsnorm_fp8=add_rmsnorm_fp8,
                           silu_mul_fp8=silu_mul_fp8, linear_fp8=linear_fp8, gemm_nt_fp8=gemm_nt_fp8, fp8_cfg=fp8_cfg, rmsnorm=rmsnorm, add_rmsnorm=add_rmsnorm, silu_mul=silu_mul,
                           embed_rmsnorm=embed_rmsnorm,
                           qk_norm_rope_kv_write=qk_norm_rope_kv_write,
                           paged_attention_decode=paged_attention_decode,
                           decode_workspace_numel=decode_workspace_numel,
                           decode_max_context=lambda cascade=True: lib.bcg_decode_max_context(int(cascade)),
                           paged_attention_prefill=paged_attention_prefill,
                           prefill_tile_rows=prefill_tile_rows,
                           sample_step=sample_step, dispatch_log=dispatch_log,
                           library=lib)
