"""Shared-prefix (cascade) decode attention on the GPU against the fp32 reference.  GPU only.

Rows of a group map the same physical leading KV blocks (what the prefix cache produces);
``decode_shared_kernel`` computes their attention over those blocks once per group into
split slot 0, ``decode_attn_kernel`` covers each row's own tokens, the combine merges both.
Covered: GQA ratios 5 / 7 / 8 and head dims 128 / 64, bf16 and fp8 KV, odd shared block
counts (the masked half chunk), groups wider than one 64-column item, rows whose own part
is a single token, ungrouped rows beside grouped ones, large batches, and a HIP graph
replayed after the tables change underneath it (the engine re-plans between bursts).
"""
import pytest
import torch

from byzantine_consensus_llm_agents_amd.engine.cascade import CascadeTables, plan_groups
from byzantine_consensus_llm_agents_amd.ops import reference as R

pytestmark = pytest.mark.gpu
F8 = torch.float8_e4m3fn


@pytest.fixture(scope="module")
def hip():
    from byzantine_consensus_llm_agents_amd.ops import get_ops
    return get_ops("hip")


def _case(gen, families, singles, NB, max_blocks, own_max=700):
    perm = (torch.randperm(NB - 1, generator=gen) + 1).tolist()
    nxt = 0

    def take(n):
        nonlocal nxt
        out = perm[nxt:nxt + n]
        nxt += n
        assert nxt <= len(perm)
        return out

    rows, lens = [], []
    for members, shared in families:
        common = take(shared)
        for i in range(members):
            own = 1 if i == 0 else int(torch.randint(1, own_max, (1,), generator=gen))
            ctx = shared * 16 + own
            rows.append(common + take((ctx + 15) // 16 - shared))
            lens.append(ctx)
    for _ in range(singles):
        ctx = int(torch.randint(1, 1200, (1,), generator=gen))
        rows.append(take((ctx + 15) // 16))
        lens.append(ctx)
    order = torch.randperm(len(rows), generator=gen).tolist()
    rows, lens = [rows[i] for i in order], [lens[i] for i in order]
    tables = torch.zeros(len(rows), max_blocks, dtype=torch.int32)
    for r, blks in enumerate(rows):
        assert len(blks) <= max_blocks
        tables[r, :len(blks)] = torch.tensor(blks, dtype=torch.int32)
    return rows, tables.cuda(), torch.tensor(lens, dtype=torch.int32, device="cuda")


def _caches(L, NB, n_kv, hd, dtype):
    k = torch.randn(L, NB, n_kv, 16, hd, device="cuda", dtype=torch.bfloat16)
    v = torch.randn(L, NB, n_kv, hd, 16, device="cuda", dtype=torch.bfloat16)
    return k.to(dtype), v.to(dtype)


def _close(a, b, atol=2e-2):
    torch.testing.assert_close(a.float(), b.float(), atol=atol, rtol=2e-2)


@pytest.mark.parametrize("kv_dtype", [torch.bfloat16, F8])
@pytest.mark.parametrize("n_q,n_kv,hd", [(40, 8, 128), (14, 2, 64), (64, 8, 128), (16, 2, 128)])
def test_cascade_decode_vs_fp32(hip, n_q, n_kv, hd, kv_dtype):
    gen = torch.Generator().manual_seed(11)
    NB, max_blocks = 4096, 128
    # 23 / 41 shared blocks: odd counts end in a masked half chunk; 30 members x G columns
    # span several 64-column items
    rows, tables, seq = _case(gen, [(30, 23), (7, 41), (3, 4), (2, 64)], singles=9, NB=NB, max_blocks=max_blocks)
    B = len(rows)
    k, v = _caches(2, NB, n_kv, hd, kv_dtype)
    q = torch.randn(B, n_q, hd, device="cuda", dtype=torch.bfloat16)
    t = CascadeTables(B, "cuda")
    groups = plan_groups(list(enumerate(rows)))
    assert len(groups) == 4
    t.upload(groups, heads_per_kv=n_q // n_kv)
    scale = hd ** -0.5
    ref = R.paged_attention(q, k, v, 1, tables, torch.arange(B + 1, dtype=torch.int32, device="cuda"), seq, scale)
    out = hip.paged_attention_decode(q, k, v, 1, tables, seq, scale, None, t)
    plain = hip.paged_attention_decode(q, k, v, 1, tables, seq, scale)
    _close(out, ref)
    _close(out, plain)
    # no groups: the same kernels with empty tables are the plain path
    t.upload([], heads_per_kv=n_q // n_kv)
    _close(hip.paged_attention_decode(q, k, v, 1, tables, seq, scale, None, t), ref)


def test_cascade_decode_large_batch_wide_groups(hip):
    """1400 rows in groups of up to 160 (800 columns: 13 items of one group per kv head)."""
    gen = torch.Generator().manual_seed(12)
    n_q, n_kv, hd, NB, max_blocks = 40, 8, 128, 32768, 96
    fams = [(160, 40), (150, 38), (120, 15), (100, 9), (90, 40), (300, 12), (200, 33), (80, 50)]
    rows, tables, seq = _case(gen, fams, singles=200, NB=NB, max_blocks=max_blocks, own_max=500)
    B = len(rows)
    k, v = _caches(1, NB, n_kv, hd, torch.bfloat16)
    q = torch.randn(B, n_q, hd, device="cuda", dtype=torch.bfloat16)
    t = CascadeTables(B, "cuda")
    t.upload(plan_groups(list(enumerate(rows))), heads_per_kv=n_q // n_kv)
    ref = R.paged_attention(q, k, v, 0, tables, torch.arange(B + 1, dtype=torch.int32, device="cuda"), seq,
                            hd ** -0.5)
    _close(hip.paged_attention_decode(q, k, v, 0, tables, seq, hd ** -0.5, None, t), ref)


def test_cascade_decode_graph_replay_after_replan(hip):
    """A captured decode (fixed workspace + table buffers) stays right when the tables are
    re-planned between replays -- with a different grouping, and with none."""
    gen = torch.Generator().manual_seed(13)
    n_q, n_kv, hd, NB, max_blocks = 40, 8, 128, 4096, 96
    rows, tables, seq = _case(gen, [(20, 21), (12, 30)], singles=8, NB=NB, max_blocks=max_blocks)
    B = len(rows)
    k, v = _caches(1, NB, n_kv, hd, torch.bfloat16)
    q = torch.randn(B, n_q, hd, device="cuda", dtype=torch.bfloat16)
    t = CascadeTables(64, "cuda")
    ws = torch.empty(hip.decode_workspace_numel(64, n_q, hd, max_blocks), dtype=torch.float32, device="cuda")
    groups = plan_groups(list(enumerate(rows)))
    t.upload(groups, heads_per_kv=5)
    ref = R.paged_attention(q, k, v, 0, tables, torch.arange(B + 1, dtype=torch.int32, device="cuda"), seq,
                            hd ** -0.5)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        hip.paged_attention_decode(q, k, v, 0, tables, seq, hd ** -0.5, ws, t)
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out = hip.paged_attention_decode(q, k, v, 0, tables, seq, hd ** -0.5, ws, t)
    for plan in (groups, [], [groups[0]], [groups[1]], groups):
        t.upload(plan, heads_per_kv=5)
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        _close(out, ref)
