"""Shared-prefix (cascade) decode tables: grouping and the semantics the HIP kernels implement.

``engine/cascade.py`` groups decode rows whose leading KV blocks are the same physical
blocks; the HIP decode attention then reads those blocks once per group.  Here (CPU):
the grouping rule, the packed device image, and -- through the fp32 emulation of the
kernels' split/merge (``reference.paged_attention_decode_cascade``) -- that attention
computed from the tables equals plain paged attention.
"""
import torch

from byzantine_consensus_llm_agents_amd.engine.cascade import (COLS_PER_ITEM, CascadeTables, MIN_SHARED_BLOCKS,
                                                               SPLIT_TOKENS, plan_groups)
from byzantine_consensus_llm_agents_amd.ops import reference as R


def make_case(gen, families, singles, max_blocks=64, NB=2048, extra=(1, 40)):
    """Rows whose tables start with a family's shared blocks then private blocks.

    families: [(members, shared blocks)], singles: rows with no sharing.
    Returns (row block lists, seq_lens)."""
    perm = (torch.randperm(NB - 1, generator=gen) + 1).tolist()
    nxt = 0

    def take(n):
        nonlocal nxt
        out = perm[nxt:nxt + n]
        nxt += n
        return out

    rows, lens = [], []
    for members, shared in families:
        common = take(shared)
        for _ in range(members):
            own = int(torch.randint(extra[0], extra[1] * 16, (1,), generator=gen))
            ctx = shared * 16 + own
            rows.append(common + take((ctx + 15) // 16 - shared))
            lens.append(ctx)
    for _ in range(singles):
        ctx = int(torch.randint(1, 600, (1,), generator=gen))
        rows.append(take((ctx + 15) // 16))
        lens.append(ctx)
    order = torch.randperm(len(rows), generator=gen).tolist()  # families interleaved over rows
    return [rows[i] for i in order], [lens[i] for i in order]


def test_plan_groups_families_and_singletons():
    gen = torch.Generator().manual_seed(0)
    rows, _ = make_case(gen, [(5, 12), (3, 7), (2, MIN_SHARED_BLOCKS - 1)], singles=6)
    groups = plan_groups(list(enumerate(rows)))
    got = sorted((len(m), s) for m, s in groups)
    assert got == [(3, 7), (5, 12)]  # the 2-row family shares too little to be worth a pass
    for members, shared in groups:
        lead = rows[members[0]]
        assert all(rows[m][:shared] == lead[:shared] for m in members)


def test_plan_groups_keeps_the_larger_saving():
    # 4 rows share 20 blocks; a 5th shares only 5 of them with the run: taking it in would
    # save 4 x 5 = 20 < 3 x 20 = 60 blocks, so it stays out (and forms no group of its own)
    base = list(range(100, 120))
    rows = [(i, base + [200 + 10 * i + j for j in range(3)]) for i in range(4)]
    rows.append((4, base[:5] + [900, 901]))
    groups = plan_groups(rows)
    assert groups == [([0, 1, 2, 3], 20)]


def test_tables_image():
    gen = torch.Generator().manual_seed(1)
    rows, _ = make_case(gen, [(30, 9), (4, 5)], singles=3)
    groups = plan_groups(list(enumerate(rows)))
    t = CascadeTables(64, "cpu")
    t.upload(groups, heads_per_kv=5)
    n_items = int(t.n_items[0])
    n_split = lambda shared: (16 * shared + SPLIT_TOKENS - 1) // SPLIT_TOKENS  # noqa: E731
    assert n_items == sum(n_split(s) * ((len(m) * 5 + COLS_PER_ITEM - 1) // COLS_PER_ITEM) for m, s in groups)
    items = t.items[:n_items].tolist()
    for g, (members, shared) in enumerate(groups):
        first, n, s, _ = t.grp_desc[g].tolist()
        assert n == len(members) and s == shared
        assert t.grp_rows[first:first + n].tolist() == members
        for m in members:
            assert int(t.kv_begin[m]) == 16 * shared and int(t.split_base[m]) == n_split(shared)
        mine = sorted((cb, sp) for gg, cb, sp, _ in items if gg == g)
        n_cb = (len(members) * 5 + COLS_PER_ITEM - 1) // COLS_PER_ITEM
        assert mine == sorted((cb, sp) for cb in range(n_cb) for sp in range(n_split(shared)))
    grouped = {m for ms, _ in groups for m in ms}
    for r in range(len(rows)):
        if r not in grouped:
            assert int(t.kv_begin[r]) == 0 and int(t.split_base[r]) == 0
    # re-planning with no groups clears everything
    t.upload([], heads_per_kv=5)
    assert int(t.n_items[0]) == 0 and int(t.kv_begin.abs().sum()) == 0


def test_cascade_attention_equals_paged_attention():
    gen = torch.Generator().manual_seed(2)
    torch.manual_seed(2)
    n_q, n_kv, hd, L, NB, max_blocks = 10, 2, 32, 2, 512, 48
    rows, lens = make_case(gen, [(14, 11), (3, 6), (5, 4)], singles=4, max_blocks=max_blocks, NB=NB, extra=(1, 12))
    B = len(rows)
    tables = torch.zeros(B, max_blocks, dtype=torch.int32)
    for r, blks in enumerate(rows):
        tables[r, :len(blks)] = torch.tensor(blks, dtype=torch.int32)
    k = torch.randn(L, NB, n_kv, 16, hd)
    v = torch.randn(L, NB, n_kv, hd, 16)
    q = torch.randn(B, n_q, hd)
    seq = torch.tensor(lens, dtype=torch.int32)
    t = CascadeTables(B, "cpu")
    t.upload(plan_groups(list(enumerate(rows))), heads_per_kv=n_q // n_kv)
    assert int(t.n_items[0]) > 0
    ref = R.paged_attention(q, k, v, 1, tables, torch.arange(B + 1, dtype=torch.int32), seq, hd ** -0.5)
    out = R.paged_attention_decode_cascade(q, k, v, 1, tables, seq, hd ** -0.5, t)
    torch.testing.assert_close(out, ref, atol=1e-5, rtol=1e-5)
