"""Shared-prefix (cascade) decode attention: which rows share KV blocks, as device tables.

With prefix caching, every agent's system prompt + chat header is computed once and its
full KV blocks are handed to every later request with the same prompt prefix -- the same
agent role in every concurrent game (SURVEY §2.3 K-ATTN-D; ``engine/engine.py`` admission).
In the driver's bench ~40 % of a decode row's context sits in such shared blocks, and the
per-row decode kernel streams them once per row: the same bytes, ~20-100 times per step.

``plan_groups`` groups the live rows whose leading physical block ids coincide;
``CascadeTables`` holds the result on the device where the decode graphs read it:

* ``kv_begin[row]``    shared tokens of the row (0: not in a group) -- the per-row kernel
                       starts there;
* ``split_base[row]``  the shared pass's splits of the row's group: its partial slots
                       0 .. split_base-1 hold the shared part, its own splits follow;
* ``grp_rows``         the members of every group, contiguous;
* ``grp_desc[g]``      (first member index in grp_rows, members, shared blocks, 0);
* ``items[i]``         (group, 64-column block, shared split of SPLIT_TOKENS tokens, 0): one
                       wave of ``decode_shared_kernel`` each;
* ``n_items``          live item count (a device scalar: graph replays read the current one).

All of it lives in ONE int32 device buffer refreshed by one async host->device copy when the
row layout changes (admission, completion, compaction) -- between decode bursts, on the
engine's stream, so a burst always sees tables that match its rows.  The result of the
attention is unchanged (the split partials merge exactly as flash-decoding's do); the torch
reference backend ignores the tables.
"""

from typing import List, Sequence, Tuple

import numpy as np
import torch

MIN_SHARED_BLOCKS = 4     # below 64 shared tokens the extra pass is not worth its launch
SPLIT_TOKENS = 128        # shared tokens per work item (a multiple of the kernel's 32-token chunk)
MAX_SHARED_SPLITS = 16    # = DEC_MAX_SHARED_SPLITS in csrc/kernels/attention.hip
MAX_SHARED_BLOCKS = MAX_SHARED_SPLITS * SPLIT_TOKENS // 16  # 2048 tokens
COLS_PER_ITEM = 64        # decode_shared_kernel: 4 MFMA column tiles of 16 per wave


def _lcp(a: Sequence[int], b: Sequence[int], limit: int) -> int:
    n = min(len(a), len(b), limit)
    i = 0
    while i < n and a[i] == b[i]:
        i += 1
    return i


def plan_groups(rows: List[Tuple[int, Sequence[int]]], min_shared: int = MIN_SHARED_BLOCKS,
                max_shared: int = MAX_SHARED_BLOCKS) -> List[Tuple[List[int], int]]:
    """Group rows by common leading block ids.

    ``rows``: (row index, the row's block ids in order).  Returns [(member rows, shared
    blocks)], every group with >= 2 members and >= ``min_shared`` blocks.  Rows are sorted by
    their block ids, so rows sharing a prefix are adjacent; a run grows while the blocks it
    saves, (members - 1) x shared, do not shrink by taking the next row in (whose common
    prefix with the run's first row may be shorter).
    """
    order = sorted(((tuple(blks[:max_shared]), row) for row, blks in rows))
    groups: List[Tuple[List[int], int]] = []
    lead, members, shared = None, [], 0

    def close():
        if len(members) >= 2 and shared >= min_shared:
            groups.append((list(members), shared))

    for blks, row in order:
        if lead is not None:
            lcp = _lcp(lead, blks, shared)
            n = len(members)
            if lcp >= min_shared and n * lcp >= (n - 1) * shared:
                members.append(row)
                shared = lcp
                continue
            close()
        lead, members, shared = blks, [row], len(blks)
    if lead is not None:
        close()
    return groups


class CascadeTables:
    """Device-resident shared-prefix tables for up to ``cap`` decode rows (see module doc)."""

    def __init__(self, cap: int, device, block_size: int = 16):
        self.cap, self.block_size = cap, block_size
        self.split_tokens = SPLIT_TOKENS
        self.max_groups = cap // 2 + 1
        self.max_items = 8 * cap + 64  # groups that would overflow it stay ungrouped
        sizes = [cap, cap, cap, 4 * self.max_groups, 4 * self.max_items, 1]
        self.buf = torch.zeros(sum(sizes), dtype=torch.int32, device=device)
        self._host = np.zeros(sum(sizes), dtype=np.int32)
        views, off = [], 0
        for n in sizes:
            views.append((off, off + n))
            off += n
        self._off = views
        b = self.buf
        self.kv_begin = b[views[0][0]:views[0][1]]
        self.split_base = b[views[1][0]:views[1][1]]
        self.grp_rows = b[views[2][0]:views[2][1]]
        self.grp_desc = b[views[3][0]:views[3][1]].view(self.max_groups, 4)
        self.items = b[views[4][0]:views[4][1]].view(self.max_items, 4)
        self.n_items = b[views[5][0]:views[5][1]]
        self.groups: List[Tuple[List[int], int]] = []
        self.shared_row_blocks = 0   # sum over grouped rows of their shared blocks (stats)

    def fill_host(self, groups: List[Tuple[List[int], int]], heads_per_kv: int) -> np.ndarray:
        """The packed int32 image of the tables for ``groups`` (CPU; what `upload` copies)."""
        h = self._host
        h[:] = 0
        (kb0, _), (sb0, _), (gr0, _), (gd0, _), (it0, _), (ni0, _) = self._off
        pos, n_items, shared_rows = 0, 0, 0
        groups = groups[:self.max_groups]
        for g, (members, shared) in enumerate(groups):
            members = [m for m in members if 0 <= m < self.cap][:self.cap - pos]
            shared = min(shared, MAX_SHARED_BLOCKS)
            if len(members) < 2 or shared <= 0:
                continue
            n_split = (shared * self.block_size + self.split_tokens - 1) // self.split_tokens
            n_cb = (len(members) * heads_per_kv + COLS_PER_ITEM - 1) // COLS_PER_ITEM
            if n_items + n_split * n_cb > self.max_items:
                continue
            for m in members:
                h[kb0 + m] = shared * self.block_size
                h[sb0 + m] = n_split
            h[gr0 + pos:gr0 + pos + len(members)] = members
            h[gd0 + 4 * g:gd0 + 4 * g + 3] = (pos, len(members), shared)
            pos += len(members)
            shared_rows += shared * len(members)
            for sp in range(n_split):  # split-major: a group's column blocks of one split adjacent
                for cb in range(n_cb):
                    h[it0 + 4 * n_items:it0 + 4 * n_items + 3] = (g, cb, sp)
                    n_items += 1
        h[ni0] = n_items
        self.groups = groups
        self.shared_row_blocks = shared_rows
        return h

    def upload(self, groups: List[Tuple[List[int], int]], heads_per_kv: int):
        """Refresh the device tables (async, stream-ordered behind the bursts already queued)."""
        host = torch.from_numpy(self.fill_host(groups, heads_per_kv).copy())
        if self.buf.device.type == "cuda":
            host = host.pin_memory()
        self.buf.copy_(host, non_blocking=True)
