"""HIP-graph capture of the full decode step (forward + guided sampling).

A decode step launches ~10 kernels per layer (GEMMs, norms, rope/KV-write,
attention + split combine, SiLU, all-reduce under TP) plus the sampler --
~400 launches for Qwen3-14B -- so eager launching is host-bound; a replay
costs one ``hipGraphLaunch``.

All graphs read and write the engine's single per-row state table
(``engine.state``): the graph of bucket ``b`` is captured over the views
``state[k][:b]``, so every bucket sees the same rows and the continuous-batching
scheduler can admit / retire / compact rows between bursts of replays without
re-capturing.  Inactive rows are parked (done, context 1 on scratch block 0).
Graphs are invalidated when the FSM table is re-allocated (its pointer is
baked into the captured sampler launch).
"""

from typing import Dict

import torch

# 32-row steps above 128: a decode step computes every row of its bucket, so the
# padding between the live rows and the bucket is wasted GEMM work (~5 % at
# 32-row steps against ~12 % at the former 64/128-row steps, B ~ 330).
# Buckets above 768 are captured only when the engine's max_batch_seqs allows them.
BUCKETS = (1, 2, 4, 8, 12, 16, 24, 32, 40, 48, 64, 80, 96, 112, 128) + tuple(range(160, 1025, 32)) + \
    tuple(range(1088, 1537, 64))
MAX_ROWS = BUCKETS[-1]


def bucket_for(n: int) -> int:
    for b in BUCKETS:
        if b >= n:
            return b
    return MAX_ROWS


class DecodeGraphs:
    def __init__(self, engine):
        self.engine = engine
        self.graphs: Dict[int, torch.cuda.CUDAGraph] = {}
        self.pool = None
        self.version = None
        self.captures = 0

    def _views(self, b: int):
        return {k: v[:b] for k, v in self.engine.state.items()}

    def _capture(self, b: int) -> torch.cuda.CUDAGraph:
        e = self.engine
        view = self._views(b)
        # capture-time replays must not disturb live rows: snapshot the state
        saved = {k: v.clone() for k, v in e.state.items()}
        if self.pool is None:
            self.pool = torch.cuda.graph_pool_handle()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(2):  # warm-up: allocator + library plans
                e.decode_step(view)
        torch.cuda.current_stream().wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, pool=self.pool):
            e.decode_step(view)
        for k, v in e.state.items():
            v.copy_(saved[k])
        torch.cuda.synchronize()
        self.captures += 1
        return graph

    def capture_all(self, max_rows: int):
        """Capture every bucket up to `max_rows` now (idle rows are parked), so no
        capture lands later in the middle of serving.  Largest first: the graphs
        share one private pool, and smaller captures then carve their
        activations out of the blocks the largest one freed (ascending order
        made every capture allocate fresh segments: 19.75 GiB for Qwen3-32B)."""
        for b in sorted((b for b in BUCKETS if b <= max_rows), reverse=True):
            if b not in self.graphs:
                self.graphs[b] = self._capture(b)

    def run_burst(self, n_rows: int) -> int:
        """Replay the bucket covering rows [0, n_rows) `poll_every` times."""
        e = self.engine
        if self.version != e.fsm.version:
            self.graphs.clear()
            # no graph references the old FSM tables any more; replays still in flight
            # finish before anything re-uses that memory (same stream, stream-ordered allocator)
            e.fsm.release_retired()
            self.version = e.fsm.version
            if e.args.precapture_graphs:
                self.capture_all(e.state["done"].shape[0])
        b = bucket_for(n_rows)
        graph = self.graphs.get(b)
        if graph is None:
            graph = self.graphs[b] = self._capture(b)
        for _ in range(e.args.poll_every):
            graph.replay()
        return e.args.poll_every
