"""Per-phase wall-clock timers and roctx ranges (the reference has none).

``PhaseTimer.phase(name)`` accumulates host wall time per phase (tokenize,
fsm_compile, prefill, sample, decode, detokenize ...).  With
``BCG_TRACE_SYNC=1`` each phase synchronises the device first so the numbers
are device-accurate; with ``BCG_ROCTX=1`` each phase is also a roctx range,
visible in ``rocprofv3 --marker-trace`` timelines.
"""

import os
import time
from collections import defaultdict
from contextlib import contextmanager

import torch

_SYNC = os.environ.get("BCG_TRACE_SYNC", "0") == "1"
_ROCTX = os.environ.get("BCG_ROCTX", "0") == "1"


class PhaseTimer:
    def __init__(self):
        self.totals = defaultdict(float)
        self.counts = defaultdict(int)

    @contextmanager
    def phase(self, name: str):
        if _SYNC and torch.cuda.is_available():
            torch.cuda.synchronize()
        if _ROCTX and torch.cuda.is_available():
            torch.cuda.nvtx.range_push(name)
        t0 = time.perf_counter()
        try:
            yield
        finally:
            if _SYNC and torch.cuda.is_available():
                torch.cuda.synchronize()
            self.totals[name] += time.perf_counter() - t0
            self.counts[name] += 1
            if _ROCTX and torch.cuda.is_available():
                torch.cuda.nvtx.range_pop()

    def summary(self):
        return {k: {"seconds": round(v, 4), "count": self.counts[k]} for k, v in sorted(self.totals.items())}

    def reset(self):
        self.totals.clear()
        self.counts.clear()
