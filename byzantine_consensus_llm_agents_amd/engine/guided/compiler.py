"""Schema -> token-level FSM tables, cached and packed into one device tensor.

``FSMRegistry.get(schema)`` returns the row base of the schema's table inside
a single ``int16 [rows, vocab]`` device tensor (``table``) plus a per-row
``dist`` vector.  A decoding sequence carries ``(fsm_base, fsm_state)``; the
sampling kernel reads ``table[fsm_base + fsm_state]`` -- so any mix of
schemas shares one batch (the fix for the reference's batch-size-1
fallback).
"""

import hashlib
import json
import threading
from dataclasses import dataclass
from typing import Dict, List, Optional

import numpy as np
import torch

from .json_schema import schema_to_dfa, validity_aware


@dataclass
class CompiledFSM:
    key: str
    next: np.ndarray     # int16 [S, V]
    dist: np.ndarray     # int16 [S]
    num_byte_states: int

    @property
    def num_states(self) -> int:
        return self.next.shape[0]


def compile_schema(schema: Dict, token_bytes: List[bytes], vocab_rows: int, max_ws: int = 4,
                   native: bool = True) -> CompiledFSM:
    dfa = schema_to_dfa(schema, max_ws=max_ws)
    key = FSMRegistry.key_of(schema)
    if native:
        from ...runtime import compile_token_fsm
        nxt, dist = compile_token_fsm(dfa.trans, dfa.accept.astype(np.uint8), token_bytes, vocab_rows)
    else:
        nxt, dist = compile_token_fsm_py(dfa.trans, dfa.accept, token_bytes, vocab_rows)
    return CompiledFSM(key, np.asarray(nxt), np.asarray(dist), dfa.num_states)


def compile_token_fsm_py(trans: np.ndarray, accept: np.ndarray, token_bytes: List[bytes], vocab_rows: int):
    """Pure-Python oracle of csrc/runtime/token_fsm.cpp (small vocabularies only)."""
    S = trans.shape[0]
    nxt = np.full((S, vocab_rows), -1, dtype=np.int16)
    for s in range(S):
        for t, tb in enumerate(token_bytes[:vocab_rows]):
            if not tb:
                continue
            cur = s
            for b in tb:
                cur = int(trans[cur, b])
                if cur < 0:
                    break
            if cur >= 0:
                nxt[s, t] = cur
    dist = np.full(S, np.iinfo(np.int16).max, dtype=np.int16)
    dist[accept.astype(bool)] = 0
    changed = True
    while changed:
        changed = False
        for s in range(S):
            row = nxt[s]
            valid = row[row >= 0]
            if valid.size:
                best = int(dist[valid].min())
                if best < np.iinfo(np.int16).max and best + 1 < dist[s]:
                    dist[s] = best + 1
                    changed = True
    return nxt, dist


class FSMRegistry:
    """Compiles schemas on first use and keeps all tables resident on the device.

    Two halves with different owners:

    * ``compile(schema)`` -- the CPU work (schema -> byte DFA -> token table), on
      any thread (the simulation threads call it from ``submit``); cached by key,
      lock-free on a hit;
    * ``install(key)`` -- copies a compiled table into the packed device tensor
      and returns its row base.  Called ONLY by the thread that launches decode
      work (the engine's scheduler), between bursts: a re-allocation can then
      never race a graph replay that still reads the old tensor, and the bases
      are assigned in the scheduler's (deterministic) admission order, so TP
      ranks agree on them.  Re-allocated tables stay alive in ``retired`` until
      the decode graphs that captured them are re-captured.
    """

    def __init__(self, token_bytes: List[bytes], vocab_rows: int, device, max_ws: int = 4,
                 native: bool = True, validity_aware_min: int = 0, ascii_text: bool = False):
        self.token_bytes = token_bytes
        # > 0: every schema is compiled in its validity-aware form (json_schema.validity_aware)
        self.validity_aware_min = validity_aware_min
        self.ascii_text = ascii_text  # ... with printable-ASCII free text (json_schema.validity_aware)
        self.vocab_rows = vocab_rows
        self.device = torch.device(device)
        self.max_ws = max_ws
        self.native = native
        self._lock = threading.Lock()
        self._bases: Dict[str, int] = {}
        self._fsms: Dict[str, CompiledFSM] = {}
        self.capacity = 0
        self.table = torch.full((1, vocab_rows), -1, dtype=torch.int16, device=self.device)
        self.dist = torch.full((1,), 0, dtype=torch.int16, device=self.device)
        self.rows = 0
        self.version = 0  # bumped whenever `table`/`dist` are re-allocated (graphs must re-capture)
        self.retired: List[tuple] = []  # old (table, dist) pairs, kept until graphs re-capture

    @staticmethod
    def key_of(schema: Dict) -> str:
        # NOT sort_keys: property order is part of the grammar (the order the JSON object's
        # fields are generated in), and the key must round-trip (json.loads) to the same
        # schema -- TP followers rebuild the FSM from it
        return json.dumps(schema, separators=(",", ":"))

    def compile(self, schema: Dict) -> str:
        """CPU compile (any thread); returns the schema key for `install`."""
        if self.validity_aware_min > 0:
            schema = validity_aware(schema, self.validity_aware_min, self.ascii_text)
        key = self.key_of(schema)
        if key in self._fsms:  # lock-free hit: entries are published fully built
            return key
        with self._lock:
            if key not in self._fsms:
                self._fsms[key] = compile_schema(schema, self.token_bytes, self.vocab_rows, self.max_ws,
                                                 self.native)
        return key

    def install(self, key: str) -> int:
        """Device rows of a compiled schema (scheduler thread only); returns the row base."""
        base = self._bases.get(key)
        if base is not None:
            return base
        fsm = self._fsms[key]
        base = self.rows
        new_rows = self.rows + fsm.num_states
        if new_rows > self.capacity:
            # geometric growth keeps re-allocations (and graph re-captures) rare
            cap = max(new_rows, 2 * self.capacity, 512)
            table = torch.full((cap, self.vocab_rows), -1, dtype=torch.int16, device=self.device)
            dist = torch.zeros((cap,), dtype=torch.int16, device=self.device)
            if self.rows:
                table[:self.rows] = self.table[:self.rows]
                dist[:self.rows] = self.dist[:self.rows]
            self.retired.append((self.table, self.dist))
            self.table, self.dist, self.capacity = table, dist, cap
            self.version += 1
        self.table[base:new_rows] = torch.from_numpy(fsm.next).to(self.device)
        self.dist[base:new_rows] = torch.from_numpy(fsm.dist).to(self.device)
        self.rows = new_rows
        self._bases[key] = base
        return base

    def release_retired(self):
        """The decode graphs were re-captured against the current table: old ones may go."""
        self.retired.clear()

    def get(self, schema: Dict) -> int:
        """compile + install in one call (single-threaded users: tests, tools)."""
        return self.install(self.compile(schema))

    def fsm(self, schema: Dict) -> CompiledFSM:
        return self._fsms[self.compile(schema)]

    def start_dist(self, base: int) -> int:
        return int(self.dist[base].item())

    def signature(self) -> str:
        return hashlib.sha1("|".join(sorted(self._bases)).encode()).hexdigest()[:12]
