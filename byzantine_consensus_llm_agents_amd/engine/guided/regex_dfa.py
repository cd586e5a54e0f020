"""Tiny byte-level regular-language toolkit: AST -> Thompson NFA -> minimal DFA.

Only what the JSON-schema compiler needs: literals, byte classes, sequence,
alternation, Kleene star and bounded repetition over the 256-byte alphabet.
The resulting DFA (``trans[S,256]``, ``accept[S]``, start state 0) is the
input of the token-level compiler (``csrc/runtime/token_fsm.cpp``).
"""

from dataclasses import dataclass
from typing import Dict, FrozenSet, List, Sequence, Tuple

import numpy as np

ALL = (1 << 256) - 1


def byte_mask(*ranges: Tuple[int, int]) -> int:
    """Bitmask with bytes lo..hi (inclusive) of every range set."""
    m = 0
    for lo, hi in ranges:
        m |= ((1 << (hi - lo + 1)) - 1) << lo
    return m


def chars_mask(chars: bytes) -> int:
    m = 0
    for c in chars:
        m |= 1 << c
    return m


# ------------------------------------------------------------------- AST
class Node:
    pass


@dataclass(frozen=True)
class Lit(Node):
    data: bytes


@dataclass(frozen=True)
class Cls(Node):
    mask: int


@dataclass(frozen=True)
class Seq(Node):
    parts: Tuple[Node, ...]


@dataclass(frozen=True)
class Alt(Node):
    options: Tuple[Node, ...]


@dataclass(frozen=True)
class Star(Node):
    body: Node


@dataclass(frozen=True)
class Rep(Node):
    body: Node
    lo: int
    hi: int  # -1 = unbounded


def seq(*parts: Node) -> Node:
    flat: List[Node] = []
    for p in parts:
        if isinstance(p, Seq):
            flat.extend(p.parts)
        elif not (isinstance(p, Lit) and not p.data):
            flat.append(p)
    return flat[0] if len(flat) == 1 else Seq(tuple(flat))


def alt(*options: Node) -> Node:
    return options[0] if len(options) == 1 else Alt(tuple(options))


def lit(s) -> Node:
    return Lit(s.encode("utf-8") if isinstance(s, str) else bytes(s))


# ------------------------------------------------------------------- NFA
class _NFA:
    def __init__(self):
        self.eps: List[List[int]] = []
        self.edges: List[List[Tuple[int, int]]] = []

    def new(self) -> int:
        self.eps.append([])
        self.edges.append([])
        return len(self.eps) - 1

    def build(self, node: Node) -> Tuple[int, int]:
        """Return (start, end) states of the fragment for ``node``."""
        if isinstance(node, Lit):
            s = cur = self.new()
            for b in node.data:
                nxt = self.new()
                self.edges[cur].append((1 << b, nxt))
                cur = nxt
            return s, cur
        if isinstance(node, Cls):
            s, e = self.new(), self.new()
            self.edges[s].append((node.mask, e))
            return s, e
        if isinstance(node, Seq):
            s, e = self.build(node.parts[0])
            for part in node.parts[1:]:
                ps, pe = self.build(part)
                self.eps[e].append(ps)
                e = pe
            return s, e
        if isinstance(node, Alt):
            s, e = self.new(), self.new()
            for opt in node.options:
                os_, oe = self.build(opt)
                self.eps[s].append(os_)
                self.eps[oe].append(e)
            return s, e
        if isinstance(node, Star):
            s, e = self.new(), self.new()
            bs, be = self.build(node.body)
            self.eps[s] += [bs, e]
            self.eps[be] += [bs, e]
            return s, e
        if isinstance(node, Rep):
            parts: List[Node] = [node.body] * node.lo
            if node.hi < 0:
                parts.append(Star(node.body))
            else:
                # (b(b(b)?)?)? -- nested optionals keep the NFA linear
                opt: Node = Lit(b"")
                for _ in range(node.hi - node.lo):
                    opt = alt(seq(node.body, opt), Lit(b""))
                parts.append(opt)
            return self.build(seq(*parts) if parts else Lit(b""))
        raise TypeError(node)


def _closure(nfa: _NFA, states) -> FrozenSet[int]:
    out = set(states)
    stack = list(states)
    while stack:
        s = stack.pop()
        for t in nfa.eps[s]:
            if t not in out:
                out.add(t)
                stack.append(t)
    return frozenset(out)


class ByteDFA:
    """Deterministic automaton over bytes; state 0 is the start state."""

    def __init__(self, trans: np.ndarray, accept: np.ndarray):
        self.trans = trans.astype(np.int32)
        self.accept = accept.astype(bool)

    @property
    def num_states(self) -> int:
        return self.trans.shape[0]

    def run(self, data: bytes, state: int = 0) -> int:
        for b in data:
            if state < 0:
                return -1
            state = int(self.trans[state, b])
        return state

    def matches(self, data: bytes) -> bool:
        s = self.run(data)
        return s >= 0 and bool(self.accept[s])


def compile_dfa(node: Node) -> ByteDFA:
    nfa = _NFA()
    start, final = nfa.build(node)
    start_set = _closure(nfa, [start])
    index: Dict[FrozenSet[int], int] = {start_set: 0}
    order = [start_set]
    rows: List[List[int]] = []
    accept: List[bool] = []
    i = 0
    while i < len(order):
        cur = order[i]
        i += 1
        accept.append(final in cur)
        edges = [(m, d) for s in cur for (m, d) in nfa.edges[s]]
        row = [-1] * 256
        if edges:
            # group bytes with identical target sets
            by_target: Dict[FrozenSet[int], List[int]] = {}
            for b in range(256):
                bit = 1 << b
                tgt = frozenset(d for m, d in edges if m & bit)
                if tgt:
                    by_target.setdefault(tgt, []).append(b)
            for tgt, bs in by_target.items():
                closed = _closure(nfa, tgt)
                if closed not in index:
                    index[closed] = len(order)
                    order.append(closed)
                for b in bs:
                    row[b] = index[closed]
        rows.append(row)
    return minimize(ByteDFA(np.array(rows, dtype=np.int32), np.array(accept)))


def minimize(dfa: ByteDFA) -> ByteDFA:
    """Moore partition refinement; also drops states that cannot reach accept."""
    n = dfa.num_states
    trans, acc = dfa.trans, dfa.accept
    # co-reachability: states from which an accept state is reachable
    live = acc.copy()
    changed = True
    while changed:
        nxt = live.copy()
        for s in range(n):
            if not nxt[s]:
                row = trans[s]
                valid = row[row >= 0]
                if valid.size and live[valid].any():
                    nxt[s] = True
        changed = bool((nxt != live).any())
        live = nxt
    t = np.where((trans >= 0) & live[np.clip(trans, 0, None)], trans, -1)
    block = np.where(live, acc.astype(np.int64), -1)
    nblocks = len(np.unique(block[block >= 0]))
    alive = np.nonzero(block >= 0)[0]
    while True:
        succ = np.where(t >= 0, block[np.clip(t, 0, None)], -1)          # [n, 256]
        sig = np.concatenate([block[:, None], succ], axis=1)[alive]
        _, inv = np.unique(sig, axis=0, return_inverse=True)
        new_block = np.full(n, -1, dtype=np.int64)
        new_block[alive] = inv.reshape(-1)
        new_n = int(inv.max()) + 1 if alive.size else 0
        block = new_block
        if new_n == nblocks:
            break
        nblocks = new_n
    # renumber so that the start state's block is 0, in BFS order
    remap = {}
    queue = [int(block[0])] if block[0] >= 0 else []
    rep = {}
    for s in range(n):
        if block[s] >= 0:
            rep.setdefault(int(block[s]), s)
    while queue:
        b = queue.pop(0)
        if b in remap:
            continue
        remap[b] = len(remap)
        for x in t[rep[b]]:
            if x >= 0 and int(block[x]) not in remap:
                queue.append(int(block[x]))
    m = max(len(remap), 1)
    out_t = np.full((m, 256), -1, dtype=np.int32)
    out_a = np.zeros(m, dtype=bool)
    for b, nb in remap.items():
        s = rep[b]
        out_a[nb] = acc[s]
        for byte, x in enumerate(t[s]):
            if x >= 0:
                out_t[nb, byte] = remap[int(block[x])]
    return ByteDFA(out_t, out_a)
