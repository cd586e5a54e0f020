"""Ordering proof of the 256x256 ping-pong GEMM's LDS ring (csrc/kernels/gemm_pp.hip), on the CPU.

The kernel's correctness rests on two orderings nothing in hardware enforces for LDS-DMA:
a half-tile must be visible (every issuing wave waited for it, then a barrier the reader
passed) before any wave reads it (RAW), and a ring slot may be refilled only after every
wave's reads of its old contents retired (WAR).  This test replays the kernel's program
order -- prologue, the four phases per K-tile, the counted `vmcnt` waits, group 1 running
one barrier behind group 0 -- for every K-tile count up to a few dozen and checks both
orderings barrier by barrier, for the shipped ring geometry and the measured variants.
Broken geometries (a lead the ring cannot hold, a wait that is too shallow) must fail.
"""
import pytest


def _program(nk, ring, lead, in_mfma, depth=None):
    """Per-half-tile facts: load phase, read phase, slot; and per-phase load presence."""
    nhalf = 4 * nk
    depth = lead - 2 if depth is None else depth  # the kernel's DEPTH
    load_phase = {n: n - lead for n in range(nhalf)}  # prologue: phases -lead..-1
    read_phase = {n: n - 1 for n in range(nhalf)}     # n = 0 is read after the prologue
    has_load = lambda p: 0 <= p + lead < nhalf         # noqa: E731  (in-loop phases)
    return nhalf, depth, load_phase, read_phase, has_load


def _check(nk, ring, lead, in_mfma, depth=None):
    nhalf, depth, load_phase, read_phase, has_load = _program(nk, ring, lead, in_mfma, depth)
    # program-order list of this wave's loads: prologue first, then the loop's phases
    issued = [n for n in range(min(lead, nhalf))]
    loads_by_phase = {p: [p + lead] for p in range(4 * nk) if has_load(p)}

    def covered_at_wait(r):
        """Half-tiles whose glds a wave has certainly completed at the wait before phase r's
        first barrier (2 glds per half-tile; vmcnt(N) = all but the N youngest)."""
        seq = list(issued)
        last = r - 1 if in_mfma else r  # loads issued among the MFMAs come after the wait
        for p in range(0, last + 1):
            seq += loads_by_phase.get(p, [])
        window = r - 1 if in_mfma else r
        full = window >= 0 and has_load(window) if window >= 0 else nhalf >= lead
        n_allowed = (2 * (depth - 1) if in_mfma else 2 * depth) if full else 0
        instrs = [n for n in seq for _ in range(2)]
        done = instrs[:max(0, len(instrs) - n_allowed)]
        return set(done)

    # prologue wait: vmcnt(2*(lead-2)) when all `lead` half-tiles were issued, else vmcnt(0)
    pro = [n for n in issued for _ in range(2)]
    n_allowed = 2 * (lead - 2) if nhalf >= lead else 0
    pro_done = set(pro[:max(0, len(pro) - n_allowed)])

    # barrier after which half-tile n is visible to everyone (-1 = the prologue barrier)
    vis = {}
    for n in range(nhalf):
        per_group = []
        for g in (0, 1):
            if n in pro_done:
                per_group.append(-1)
                continue
            r = next((r for r in range(4 * nk) if n in covered_at_wait(r)), None)
            assert r is not None, f"half-tile {n} never waited for"
            per_group.append(2 * r + g)  # the wait precedes group g's pre-barrier of phase r
        vis[n] = max(per_group)

    for n in range(nhalf):
        q = read_phase[n]
        for g in (0, 1):
            start = -1 if q < 0 else 2 * q - 1 + g  # barrier a group-g wave passed before reading
            if q < 0:
                start = -1
            assert vis[n] <= start, f"RAW: half-tile {n} read in phase {q} by group {g} before visible"
        # WAR: the slot's previous occupant n - ring must be fully read before this load issues
        prev = n - ring
        if prev >= 0:
            retired = 2 * read_phase[prev] + 2  # every wave past group 1's post-barrier
            p = load_phase[n]
            for g in (0, 1):
                issue_after = 2 * p + g if in_mfma else 2 * p - 1 + g
                assert issue_after >= retired, f"WAR: slot {n % ring} refilled in phase {p} by group {g}"
        else:
            assert load_phase[n] < 0 or n < ring


@pytest.mark.parametrize("nk", [1, 2, 3, 4, 5, 8, 13, 20])
@pytest.mark.parametrize("ring,lead,in_mfma", [(10, 9, 1), (10, 9, 0), (8, 7, 1), (8, 6, 0), (8, 6, 1)])
def test_pp_ring_orderings_hold(nk, ring, lead, in_mfma):
    _check(nk, ring, lead, in_mfma)


@pytest.mark.parametrize("ring,lead,in_mfma", [(8, 8, 0), (7, 8, 1)])
def test_pp_ring_rejects_a_lead_the_ring_cannot_hold(ring, lead, in_mfma):
    # loads in the read turn need RING >= LEAD + 1; among the MFMAs (one barrier later) RING >= LEAD
    with pytest.raises(AssertionError, match="WAR"):
        _check(8, ring, lead, in_mfma)


@pytest.mark.parametrize("in_mfma", [0, 1])
def test_pp_ring_rejects_a_too_shallow_wait(in_mfma):
    # waits that leave one phase more of loads in flight (DEPTH = LEAD - 1) read too early
    with pytest.raises(AssertionError, match="RAW"):
        _check(8, 10, 9, in_mfma, depth=8)
