"""The SHIPPED GEMM dispatch at real model shapes against fp32 references.  GPU only.

* every entry of ``engine/tuned/hand_gemm.json`` -- each (M, N, K, epilogue) with the
  (tile, split-K) the table picked, or the library path (``F.linear`` / the
  ``residual.addmm_`` epilogue) where it kept hipBLASLt -- through the same ops the
  decoder calls (``linear`` / ``linear_silu`` / ``linear_residual``), compared with
  fp32 ``F.linear`` (+ SiLU*mul / + residual);
* split-K hand GEMMs captured into HIP graphs of several buckets, replayed smallest
  first (the order the engine's ramp-up replays them) against the fp32 reference;
* a 2-layer decoder with Qwen3-14B's real dimensions (random weights): the HIP
  forward of one 16384-token prefill chunk and of decode buckets 16 and 512, against
  the fp32 torch forward of the same weights.

The table entries each test touched are printed (``-s`` / the GPU log shows them).
"""
import json
import os
from collections import defaultdict

import pytest
import torch

pytestmark = pytest.mark.gpu

TABLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "byzantine_consensus_llm_agents_amd",
                     "engine", "tuned", "hand_gemm.json")


def _entries():
    with open(TABLE) as fh:
        choice = json.load(fh)["choice"]
    by_shape = defaultdict(list)
    for key, ch in choice.items():
        m, n, k, e = map(int, key.split(","))
        by_shape[(n, k, e)].append((m, tuple(ch) if isinstance(ch, list) else (int(ch), 1)))
    return {s: sorted(v) for s, v in by_shape.items()}


ENTRIES = _entries()


@pytest.fixture(scope="module")
def hip():
    from byzantine_consensus_llm_agents_amd.ops import get_ops
    ops = get_ops("hip")
    plan = ops.gemm_plan
    saved = (plan.mode, plan.force_split)
    plan.mode, plan.force_split = "1", 1  # the shipped table
    yield ops
    plan.mode, plan.force_split = saved


def _err(out, ref):
    out, ref = out.float(), ref.float()
    return (out - ref).abs().max().item() / max(1e-6, ref.abs().max().item())


@pytest.mark.parametrize("shape", sorted(ENTRIES), ids=lambda s: f"N{s[0]}_K{s[1]}_epi{s[2]}")
def test_shipped_table_entries(hip, shape):
    N, K, epi = shape
    gen = torch.Generator(device="cuda").manual_seed(N + K + epi)
    w = (torch.randn(N, K, device="cuda", generator=gen) * K ** -0.5).to(torch.bfloat16)
    touched = []
    for M, choice in ENTRIES[shape]:
        x = torch.randn(M, K, device="cuda", generator=gen).to(torch.bfloat16)
        assert hip.gemm_plan.choose(M, N, K, epi) == (choice if choice[0] >= 0 else None) or choice[0] < 0
        ref = x.float() @ w.float().t()
        if epi == 0:
            out = hip.linear(x, w)
        elif epi == 1:
            out = hip.linear_silu(x, w)
            I = N // 2
            ref = torch.nn.functional.silu(ref[:, :I]) * ref[:, I:]
        else:
            res = torch.randn(M, N, device="cuda", generator=gen).to(torch.bfloat16)
            ref = ref + res.float()
            out = hip.linear_residual(x, w, res)
            assert out.data_ptr() == res.data_ptr()  # in place
        torch.cuda.synchronize()
        e = _err(out, ref)
        touched.append(f"{M}:{'lib' if choice[0] < 0 else '%dx%d' % choice}:{e:.1e}")
        assert e < 2e-2, (M, choice, e)
        del x, ref, out
    print(f"[table] N={N} K={K} epi={epi} entries(M:choice:err) " + " ".join(touched))


def test_split_k_graphs_replay_small_bucket_first(hip):
    """Split-K hand GEMMs in graphs captured largest-first, replayed smallest-first and
    repeatedly: every replay must reduce every tile (the arrival counters are allocated
    before capture and reset by each tile's last arriver)."""
    plan = hip.gemm_plan
    K, N = 5120, 5120
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    buckets = (512, 64, 8)
    xs = {m: torch.randn(m, K, device="cuda").to(torch.bfloat16) for m in buckets}
    outs, graphs = {}, {}
    cfgs = {512: (7, 3), 64: (1, 4), 8: (6, 6)}  # (tile, split): split-K in every bucket
    for m in buckets:
        assert plan.supported(cfgs[m][0], m, N, K, 0, cfgs[m][1])
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):  # warm-up outside capture
        for m in buckets:
            hip.gemm_nt(xs[m], w, cfgs[m])
    torch.cuda.current_stream().wait_stream(side)
    pool = torch.cuda.graph_pool_handle()
    for m in buckets:  # largest first, as DecodeGraphs.capture_all
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, pool=pool):
            outs[m] = hip.gemm_nt(xs[m], w, cfgs[m])
        graphs[m] = g
    for rep in range(3):
        for m in reversed(buckets):
            outs[m].zero_()
            graphs[m].replay()
            torch.cuda.synchronize()
            assert _err(outs[m], xs[m].float() @ w.float().t()) < 2e-2, (rep, m)


def _qwen3_14b_2layer():
    import dataclasses

    from byzantine_consensus_llm_agents_amd.models.config import get_model_config
    from byzantine_consensus_llm_agents_amd.models.transformer import DecoderModel
    from byzantine_consensus_llm_agents_amd.ops import get_ops
    cfg = dataclasses.replace(get_model_config("qwen3-14b"), num_layers=2)
    mh = DecoderModel(cfg, get_ops("hip"), "cuda", torch.bfloat16)
    mh.init_random(seed=11, std=0.02)
    mt = DecoderModel(cfg, get_ops("torch"), "cuda", torch.float32)
    mt.load_hf_state_dict(mh.hf_state_dict())
    return cfg, mh, mt


def _close_logits(out, ref, what):
    out, ref = out.float(), ref.float()
    rel = ((out - ref).norm() / ref.norm()).item()
    mx = (out - ref).abs().max().item() / ref.abs().max().item()
    cos = torch.nn.functional.cosine_similarity(out, ref, dim=-1).min().item()
    print(f"[decoder] {what}: rel_l2={rel:.2e} max_rel={mx:.2e} min_cos={cos:.5f}")
    assert rel < 2e-2 and mx < 5e-2 and cos > 0.999, (what, rel, mx, cos)


def test_qwen3_14b_shaped_decoder_vs_fp32(hip):
    """Real Qwen3-14B dimensions (2 layers): prefill chunk M = 16384, decode M = 16 and 512."""
    from byzantine_consensus_llm_agents_amd.models.batch import alloc_kv, prefill_batch
    from byzantine_consensus_llm_agents_amd.models.transformer import AttnMeta
    cfg, mh, mt = _qwen3_14b_2layer()
    n_seq, plen, bs = 16, 1024, 16
    gen = torch.Generator().manual_seed(5)
    seqs = [torch.randint(0, cfg.vocab_size, (plen,), generator=gen).tolist() for _ in range(n_seq)]
    tokens, meta, nblk = prefill_batch(seqs, bs, device="cuda")
    assert tokens.numel() == 16384
    NB = nblk + 512 + 1
    kv_h, kv_t = alloc_kv(mh, NB, bs), alloc_kv(mt, NB, bs)
    out_h = mh.forward(tokens, meta, *kv_h)
    out_t = mt.forward(tokens, meta, *kv_t)
    _close_logits(out_h, out_t, "prefill chunk M=16384")
    for B in (16, 512):
        # row r continues sequence r % 16 with its own token in a private block
        rows = torch.arange(B)
        tables = torch.zeros(B, plen // bs + 1, dtype=torch.int32)
        tables[:, :plen // bs] = meta.block_tables.cpu()[rows % n_seq, :plen // bs]
        tables[:, plen // bs] = nblk + rows.to(torch.int32)
        pos = torch.full((B,), plen, dtype=torch.int32)
        slots = tables[:, plen // bs] * bs
        dmeta = AttnMeta(positions=pos.cuda(), slots=slots.to(torch.int32).cuda(), block_tables=tables.cuda(),
                         seq_lens=torch.full((B,), plen + 1, dtype=torch.int32, device="cuda"), decode=True)
        toks = torch.randint(0, cfg.vocab_size, (B,), generator=gen, dtype=torch.int32).cuda()
        lh = mh.forward(toks, dmeta, *kv_h)
        lt = mt.forward(toks, dmeta, *kv_t)
        _close_logits(lh, lt, f"decode M={B}")
