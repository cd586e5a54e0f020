"""HIP-graph capture of the full decode step (forward + guided sampling).

One graph per batch bucket.  A decode step launches ~10 kernels per layer
(GEMMs, norm, rope/KV-write, attention + combine, SiLU, all-reduce under TP)
plus the sampler -- ~400 launches for Qwen3-14B -- so eager launching would
be host-bound; a replay costs one ``hipGraphLaunch``.  All per-row state lives
in static device buffers, the sampler advances it in place, and the host
only polls the ``done`` flags every ``poll_every`` replays.

Padding rows of a bucket are marked done and point at the scratch KV block 0.
Graphs are invalidated when the FSM table is re-allocated (its pointer is
baked into the captured sampler launch).
"""

from typing import Dict

import torch

BUCKETS = (1, 2, 4, 8, 12, 16, 24, 32, 40, 48, 64, 80, 96, 128, 160, 192, 224, 256, 320, 384, 448, 512)
OUT_WIDTH = 1024  # max tokens per sequence handled by the graph path


class DecodeGraphs:
    def __init__(self, engine):
        self.engine = engine
        self.graphs: Dict[int, tuple] = {}
        self.pool = None
        self.version = None
        self.captures = 0

    def _bucket(self, B: int) -> int:
        for b in BUCKETS:
            if b >= B:
                return b
        return -1

    def _static(self, Bb: int) -> Dict[str, torch.Tensor]:
        e = self.engine
        dev = e.device
        z = lambda: torch.zeros(Bb, dtype=torch.int32, device=dev)  # noqa: E731
        st = {"block_tables": torch.zeros(Bb, e.max_blocks_per_seq, dtype=torch.int32, device=dev),
              "seq_lens": torch.ones(Bb, dtype=torch.int32, device=dev),
              "fsm_base": torch.full((Bb,), -1, dtype=torch.int32, device=dev),
              "fsm_state": z(), "gen_count": z(), "max_new": torch.ones(Bb, dtype=torch.int32, device=dev),
              "temperature": torch.zeros(Bb, dtype=torch.float32, device=dev), "row_keys": z(),
              "done": torch.ones(Bb, dtype=torch.int32, device=dev), "next_tokens": z(),
              "out_tokens": torch.zeros(Bb, OUT_WIDTH, dtype=torch.int32, device=dev)}
        return st

    def _capture(self, Bb: int):
        e = self.engine
        st = self._static(Bb)
        if self.pool is None:
            self.pool = torch.cuda.graph_pool_handle()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(2):  # warm-up: allocator + library plans
                e.decode_step(st)
        torch.cuda.current_stream().wait_stream(side)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, pool=self.pool):
            e.decode_step(st)
        torch.cuda.synchronize()
        self.captures += 1
        return graph, st

    def run(self, st: Dict[str, torch.Tensor], B: int, max_new: int) -> int:
        e = self.engine
        Bb = self._bucket(B)
        if Bb < 0 or max_new > OUT_WIDTH:
            return self._eager(st, max_new)
        if self.version != e.fsm.version:
            self.graphs.clear()
            self.version = e.fsm.version
        if Bb not in self.graphs:
            self.graphs[Bb] = self._capture(Bb)
        graph, s = self.graphs[Bb]
        # load this wave into the static buffers (rows >= B stay padding)
        s["done"].fill_(1)
        s["seq_lens"].fill_(1)
        s["block_tables"].zero_()
        s["fsm_base"].fill_(-1)
        for key in ("block_tables", "seq_lens", "fsm_base", "fsm_state", "gen_count", "max_new",
                    "temperature", "row_keys", "done", "next_tokens"):
            s[key][:B].copy_(st[key])
        s["out_tokens"][:B, :max_new].copy_(st["out_tokens"])
        done_view = s["done"][:B]
        poll = e.args.poll_every
        steps = 0
        for i in range(1, max_new):
            if i % poll == 1 and bool(done_view.all()):
                break
            graph.replay()
            steps += 1
        for key in ("gen_count", "done", "seq_lens", "fsm_state"):
            st[key].copy_(s[key][:B])
        st["out_tokens"].copy_(s["out_tokens"][:B, :max_new])
        return steps

    def _eager(self, st, max_new: int) -> int:
        e = self.engine
        steps = 0
        for i in range(1, max_new):
            if i % e.args.poll_every == 1 and bool(st["done"].all()):
                break
            e.decode_step(st)
            steps += 1
        return steps
