"""One-shot / two-shot all-reduce over xGMI peer memory (``csrc/kernels/allreduce.hip``).

The reference's TP collectives are NCCL all-reduces inside vLLM
(``bcg/vllm_agent.py:131,139-142``; SURVEY.md §2.2, §2.3 K-COLL).  On an
MI355X node every GPU has a direct xGMI link to each of the other seven, so a
ring (RCCL's default) is per-link bound and pays n-1 latency hops.  Decode
messages are small -- ``[B, hidden]`` bf16, 10-2000 KiB -- so here each rank
maps its TP peers' buffers once (``hipIpcGetMemHandle`` exchanged over the
process group) and a single kernel does the whole collective:

* one-shot (``<= oneshot_max`` bytes): every rank pulls the full message from
  every peer and reduces locally -- one hop, all links busy at once;
* two-shot (up to ``cap_bytes``): reduce-scatter + all-gather through the
  peers' buffers, ``2(n-1)/n`` of the message per rank;
* larger messages (prefill chunks) and anything that is not contiguous bf16
  go to RCCL (``torch.distributed.all_reduce``).

Both kernels are graph-capturable (the call epoch lives in device memory) and
give bitwise-identical results on every rank (fixed summation order).
``LocalRanks`` builds the same kernels over buffers of ONE process -- the
in-process multi-stream harness the GPU tests use on a one-GPU box.
"""

import ctypes
from typing import List, Optional

import torch

ONESHOT_MAX = 1 << 20          # bytes: one-shot below, two-shot above
DEFAULT_CAP = 32 << 20         # bytes per message handled by the custom kernels
DECODE_FLOOR = 8 << 20         # bytes: messages this small always stay on the kernels (decode graphs)
THREADS = 512


def choose_mode(nbytes: int, world: int, oneshot_max: int = ONESHOT_MAX) -> int:
    """1 = one-shot, 2 = two-shot (world 8 halves the one-shot limit: 7 full reads per rank)."""
    limit = oneshot_max if world <= 4 else oneshot_max // 2
    return 1 if nbytes <= limit else 2


def pick_thresholds(sizes: List[int], t_one: List[float], t_two: List[float], t_rccl: List[float],
                    cap_bytes: int):
    """Routing limits from a measured table (bytes -> us per call, identical on every rank).

    Returns ``(oneshot_limit, route_max)``: one-shot up to the largest measured size at which it
    still beats two-shot (0: two-shot from the smallest size on), the custom kernels up to the
    largest measured size at which the kernel the routing actually picks there (one-shot up to
    ``oneshot_limit``, two-shot above) beats RCCL (RCCL beyond; ``cap_bytes`` when it wins
    everywhere).  Both limits are measured sizes (no extrapolation), and only a prefix of wins
    counts: above the first size where a method loses, the other one is used.
    """
    oneshot_limit = 0
    for nb, a, b in zip(sizes, t_one, t_two):
        if a > b:
            break
        oneshot_limit = nb
    route_max = 0
    for nb, a, b, r in zip(sizes, t_one, t_two, t_rccl):
        if (a if nb <= oneshot_limit else b) > r:
            break
        route_max = nb
    if route_max == sizes[-1]:
        route_max = cap_bytes
    return oneshot_limit, route_max


def choose_blocks(nbytes: int, world: int, mode: int, max_blocks: int = 128) -> int:
    """Workgroups per call: ~2 16-B vectors per thread per block, capped at `max_blocks`."""
    nvec = max(1, nbytes // 16)
    per_block = THREADS * 2
    if mode == 2:
        nvec = (nvec + world - 1) // world
    return int(max(1, min(max_blocks, (nvec + per_block - 1) // per_block)))


def _lib():
    from ..ops.hip import load_library
    lib = load_library()
    P, c_int, c_int64, c_double = ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_int64, ctypes.c_double
    vp = ctypes.c_void_p
    sig = {"bcg_ar_limits": [ctypes.POINTER(c_int)] * 3,
           "bcg_ar_alloc": [c_int64, P, P],
           "bcg_ar_free": [vp],
           "bcg_ar_ipc_handle_size": [],
           "bcg_ar_ipc_handle": [vp, vp],
           "bcg_ar_ipc_open": [vp, P],
           "bcg_ar_ipc_close": [vp],
           "bcg_ar_take_error": [vp],
           "bcg_ar_error_async": [vp, vp, vp],
           "bcg_ar_set_error": [vp],
           "bcg_ar_allreduce": [P, P, c_int, c_int, vp, vp, c_int64, c_int64, c_int, c_int, c_double, vp],
           "bcg_ar_allreduce_addnorm": [P, P, c_int, c_int, vp, vp, vp, vp, c_int, c_int, ctypes.c_float,
                                        c_int64, c_int, c_double, c_int, vp]}
    for name, argtypes in sig.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = c_int
    return lib


class _Rank:
    """One rank's view: pointer tables of every rank's buffers + the launch."""

    def __init__(self, lib, rank: int, world: int, data: List[int], sig: List[int], cap_bytes: int,
                 oneshot_max: int, timeout_s: float):
        self.lib, self.rank, self.world = lib, rank, world
        self.cap_bytes, self.oneshot_max, self.timeout_s = cap_bytes, oneshot_max, timeout_s
        self._data = (ctypes.c_void_p * world)(*data)
        self._sig = (ctypes.c_void_p * world)(*sig)
        mr, mb, sb = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        lib.bcg_ar_limits(ctypes.byref(mr), ctypes.byref(mb), ctypes.byref(sb))
        if world > mr.value or world & (world - 1):
            raise ValueError(f"custom all-reduce supports power-of-two groups of <= {mr.value} ranks")
        self.max_blocks = mb.value
        self.calls = {1: 0, 2: 0}
        self.route_max = cap_bytes   # messages routed to the kernels (RCCL above); calibrate() may lower it
        self.capture_route_max = cap_bytes  # the same inside a HIP-graph capture (decode): >= DECODE_FLOOR
        self.oneshot_limit = None    # measured one-shot limit (None: the choose_mode rule)
        self.addnorm_oneshot_limit = None  # ... of the fused all-reduce + add + RMSNorm kernels
        self.calibration = None

    def can(self, x: torch.Tensor) -> bool:
        n = x.numel()
        if not (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and n > 0 and n % 8 == 0
                and 2 * n <= self.cap_bytes):
            return False
        # eager calls (prefill) follow the measurement; captured calls (decode graphs) stay on the
        # kernels up to DECODE_FLOOR whatever RCCL measured (an RCCL call inside a captured step
        # is a path this build does not test)
        return 2 * n <= self.route_max or (2 * n <= self.capture_route_max
                                           and torch.cuda.is_current_stream_capturing())

    def all_reduce_(self, x: torch.Tensor, out: Optional[torch.Tensor] = None, stream=None,
                    mode: Optional[int] = None) -> torch.Tensor:
        """In-place (or into `out`) sum over the group, on the current (or given) HIP stream.
        `mode` (1 = one-shot, 2 = two-shot) overrides the routing rule (calibration)."""
        if not self.can(x):
            raise ValueError("custom all-reduce: need contiguous bf16 on the GPU, numel % 8 == 0, <= cap")
        out = x if out is None else out
        nbytes = 2 * x.numel()
        if mode is None:
            mode = (choose_mode(nbytes, self.world, self.oneshot_max) if self.oneshot_limit is None
                    else 1 if nbytes <= self.oneshot_limit else 2)
        blocks = choose_blocks(nbytes, self.world, mode, self.max_blocks)
        s = (stream or torch.cuda.current_stream()).cuda_stream
        rc = self.lib.bcg_ar_allreduce(self._data, self._sig, self.rank, self.world,
                                       ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                       x.numel(), self.cap_bytes, mode, blocks, self.timeout_s,
                                       ctypes.c_void_p(s))
        if rc != 0:
            raise RuntimeError(f"bcg_ar_allreduce launch failed (rc={rc})")
        self.calls[mode] += 1
        return out

    def calibrate(self, group, sizes: Optional[List[int]] = None, iters: int = 20, route: bool = True,
                  hidden: Optional[int] = None) -> dict:
        """Measure one-shot, two-shot and RCCL (``dist.all_reduce`` on `group`) on this group's
        own links at a few message sizes and set the routing limits from the table
        (``pick_thresholds``).  Collective over the group; the timings are max-reduced first, so
        every rank routes identically.  Replaces the built-in guesses (``ONESHOT_MAX``, halved at
        8 ranks; the buffer cap) with what this node's xGMI topology measures.  ``route=False``
        keeps the kernels' range (gloo groups chunk large messages through them).  With `hidden`
        the fused all-reduce + add + RMSNorm kernels are timed too, on [nb / 2 / hidden, hidden]
        rows, and their own one-shot limit routes ``all_reduce_add_rmsnorm``.

        Captured messages up to ``DECODE_FLOOR`` stay on the kernels whatever RCCL measures
        (``capture_route_max``): the decode graphs capture these calls, and an RCCL call inside a
        captured step is a path this build does not test.  Eager calls follow the measured
        ``route_max``; both are reported."""
        import torch.distributed as dist
        sizes = sizes or [nb for nb in (64 << 10, 256 << 10, 1 << 20, 4 << 20, 16 << 20) if nb <= self.cap_bytes]
        dev = torch.device("cuda", torch.cuda.current_device())
        table = torch.zeros(5, len(sizes), dtype=torch.float64, device=dev)
        # the fused kernels are timed only where they run at every calibrated size (H <= 8192);
        # a wider model keeps RCCL / all-reduce + add_rmsnorm (addnorm_oneshot_limit stays None)
        fused = bool(hidden) and all(
            self.can_addnorm(torch.empty(max(1, nb // (2 * hidden)), hidden, dtype=torch.bfloat16, device=dev))
            for nb in sizes)
        for i, nb in enumerate(sizes):
            x = torch.zeros(nb // 2, dtype=torch.bfloat16, device=dev)
            fns = [lambda: self.all_reduce_(x, mode=1), lambda: self.all_reduce_(x, mode=2),
                   lambda: dist.all_reduce(x, group=group)]
            if fused:
                rows = max(1, nb // (2 * hidden))
                xa = torch.zeros(rows, hidden, dtype=torch.bfloat16, device=dev)
                ra, wa = torch.zeros_like(xa), torch.ones(hidden, dtype=torch.bfloat16, device=dev)
                fns += [lambda: self.all_reduce_add_rmsnorm(xa, ra, wa, 1e-6, mode=1),
                        lambda: self.all_reduce_add_rmsnorm(xa, ra, wa, 1e-6, mode=2)]
            for m, fn in enumerate(fns):
                fn()
                torch.cuda.synchronize()
                dist.barrier(group=group)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(iters):
                    fn()
                b.record()
                b.synchronize()
                table[m, i] = a.elapsed_time(b) * 1e3 / iters
        dist.all_reduce(table, op=dist.ReduceOp.MAX, group=group)
        t = table.cpu().tolist()
        self.oneshot_limit, route_max = pick_thresholds(sizes, t[0], t[1], t[2], self.cap_bytes)
        capture_route_max = max(route_max, min(self.cap_bytes, DECODE_FLOOR))
        if route:
            self.route_max, self.capture_route_max = route_max, capture_route_max
        if fused:
            self.addnorm_oneshot_limit = pick_thresholds(sizes, t[3], t[4], t[2], self.cap_bytes)[0]
        self.calls = {1: 0, 2: 0}
        self.calibration = {"sizes": sizes, "oneshot_us": t[0], "twoshot_us": t[1], "rccl_us": t[2],
                            "oneshot_limit": self.oneshot_limit, "route_max": route_max,
                            "capture_route_max": capture_route_max}
        if fused:
            self.calibration.update(addnorm_oneshot_us=t[3], addnorm_twoshot_us=t[4],
                                    addnorm_oneshot_limit=self.addnorm_oneshot_limit, hidden=hidden)
        return self.calibration

    def error_async(self, host: torch.Tensor, stream) -> None:
        """Queue a copy of this rank's error word into pinned int32 `host[0]` on `stream`."""
        if self.lib.bcg_ar_error_async(self._sig[self.rank], ctypes.c_void_p(host.data_ptr()),
                                       ctypes.c_void_p(stream.cuda_stream)) != 0:
            raise RuntimeError("bcg_ar_error_async failed")

    def set_error(self) -> None:
        """Mark this rank's group broken (tests of the timeout path)."""
        if self.lib.bcg_ar_set_error(self._sig[self.rank]) != 0:
            raise RuntimeError("bcg_ar_set_error failed")

    def can_addnorm(self, x: torch.Tensor) -> bool:
        return (self.can(x) and x.dim() == 2 and x.shape[1] % 8 == 0 and x.shape[1] <= THREADS * 16)

    def all_reduce_add_rmsnorm(self, x: torch.Tensor, residual: torch.Tensor, w: torch.Tensor, eps: float,
                               stream=None, mode: Optional[int] = None) -> torch.Tensor:
        """residual <- residual + sum_ranks(x); returns rmsnorm(residual) * w -- one kernel, one-shot
        up to the fused kernels' own measured limit (``calibrate(hidden=...)``), two-shot above
        (rows split over the ranks; identical bits)."""
        if not self.can_addnorm(x):
            raise ValueError("fused all-reduce + RMSNorm: contiguous bf16 [rows, H<=8192], within the cap")
        rows, H = x.shape
        if not (residual.shape == x.shape and residual.is_contiguous() and residual.dtype == torch.bfloat16
                and w.shape == (H,) and w.dtype == torch.bfloat16):
            raise ValueError("fused all-reduce + RMSNorm: residual [rows, H] bf16, weight [H] bf16")
        nbytes = 2 * x.numel()
        if mode is None:
            limit = self.addnorm_oneshot_limit
            mode = (choose_mode(nbytes, self.world, self.oneshot_max) if limit is None
                    else 1 if nbytes <= limit else 2)
        h = torch.empty_like(x)
        per = rows if mode == 1 else -(-rows // self.world)
        blocks = int(max(1, min(self.max_blocks, per)))
        s = (stream or torch.cuda.current_stream()).cuda_stream
        rc = self.lib.bcg_ar_allreduce_addnorm(self._data, self._sig, self.rank, self.world,
                                               ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(residual.data_ptr()),
                                               ctypes.c_void_p(w.data_ptr()), ctypes.c_void_p(h.data_ptr()), rows,
                                               H, float(eps), self.cap_bytes, blocks, self.timeout_s, mode,
                                               ctypes.c_void_p(s))
        if rc != 0:
            raise RuntimeError(f"bcg_ar_allreduce_addnorm launch failed (rc={rc})")
        key = 3 if mode == 1 else 4
        self.calls[key] = self.calls.get(key, 0) + 1
        return h

    def take_error(self) -> bool:
        """True if a barrier of this rank timed out since the last check (synchronising)."""
        rc = self.lib.bcg_ar_take_error(self._sig[self.rank])
        if rc < 0:
            raise RuntimeError("bcg_ar_take_error failed")
        return rc == 1


def _alloc(lib, cap_bytes: int):
    d, s = ctypes.c_void_p(), ctypes.c_void_p()
    if lib.bcg_ar_alloc(cap_bytes, ctypes.byref(d), ctypes.byref(s)) != 0:
        raise RuntimeError("custom all-reduce: buffer allocation failed")
    return d.value, s.value


class XGMIAllReduce(_Rank):
    """Custom all-reduce of one TP group (one process per GPU, IPC-mapped peer buffers).

    The constructor never leaves a peer waiting: a rank whose allocation, handle export or
    peer mapping fails records why in ``error`` and still takes part in the handle exchange and
    the closing barrier.  ``establish`` (below) agrees on the outcome over the whole group and
    falls back to RCCL when any rank failed.  ``fault="ipc"`` injects a mapping failure on the
    group's last rank (tests of that fallback)."""

    def __init__(self, group, cap_bytes: int = DEFAULT_CAP, oneshot_max: int = ONESHOT_MAX,
                 timeout_s: float = 30.0, fault: Optional[str] = None):
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        self.error: Optional[str] = None
        self._own, self._opened, self.lib = None, [], None
        mine = None
        try:
            lib = self.lib = _lib()
            d, s = _alloc(lib, cap_bytes)
            self._own = (d, s)
            hsz = lib.bcg_ar_ipc_handle_size()
            hd, hs = ctypes.create_string_buffer(hsz), ctypes.create_string_buffer(hsz)
            if lib.bcg_ar_ipc_handle(ctypes.c_void_p(d), hd) or lib.bcg_ar_ipc_handle(ctypes.c_void_p(s), hs):
                raise RuntimeError("hipIpcGetMemHandle failed")
            mine = (hd.raw, hs.raw)
        except Exception as exc:  # noqa: BLE001 -- reported through `error`, agreed by establish()
            self.error = f"export: {exc}"
        handles = [None] * world
        dist.all_gather_object(handles, mine, group=group)
        data, sig = [], []
        if self.error is None:
            try:
                for r, h in enumerate(handles):
                    if h is None:
                        raise RuntimeError(f"rank {r} exported no handle")
                    if r == rank:
                        data.append(self._own[0])
                        sig.append(self._own[1])
                        continue
                    if fault == "ipc" and rank == world - 1:
                        raise RuntimeError(f"injected hipIpcOpenMemHandle failure (rank {r}'s buffers)")
                    pd, ps = ctypes.c_void_p(), ctypes.c_void_p()
                    if lib.bcg_ar_ipc_open(ctypes.create_string_buffer(h[0], hsz), ctypes.byref(pd)):
                        raise RuntimeError(f"hipIpcOpenMemHandle of rank {r} failed")
                    self._opened.append(pd.value)
                    if lib.bcg_ar_ipc_open(ctypes.create_string_buffer(h[1], hsz), ctypes.byref(ps)):
                        raise RuntimeError(f"hipIpcOpenMemHandle of rank {r} failed")
                    self._opened.append(ps.value)
                    data.append(pd.value)
                    sig.append(ps.value)
                super().__init__(lib, rank, world, data, sig, cap_bytes, oneshot_max, timeout_s)
            except Exception as exc:  # noqa: BLE001
                self.error = f"ipc: {exc}"
        dist.barrier(group=group)  # every peer mapped (or failed) before anyone launches

    def close(self):
        if self._own is None and not self._opened:
            return
        torch.cuda.synchronize()
        for p in self._opened:
            self.lib.bcg_ar_ipc_close(ctypes.c_void_p(p))
        for p in self._own or ():
            self.lib.bcg_ar_free(ctypes.c_void_p(p))
        self._own, self._opened = None, []


def cross_check(custom, group, device, fault: Optional[str] = None) -> Optional[str]:
    """One-shot and two-shot all-reduce of a rank-dependent tensor against the process group's
    own ``dist.all_reduce`` (small integers: exact in bf16, so the results must be bitwise equal).
    Returns None when both agree, else what differed.  ``fault="mismatch"`` perturbs the custom
    result on the group's last rank (tests of the fallback).  Every rank runs every collective
    whatever it found (an early return would leave its peers waiting in the next one)."""
    import torch.distributed as dist
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    found = None
    for mode, n in ((1, 4096), (2, min(custom.cap_bytes // 2, 1 << 20) // 8 * 8)):
        x = ((torch.arange(n, device=device) % 7) + rank + 1).to(torch.bfloat16)
        ref = x.clone()
        dist.all_reduce(ref, group=group)
        got = custom.all_reduce_(x.clone(), mode=mode)
        if fault == "mismatch" and rank == world - 1:
            got[n // 2] += 1
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        if not torch.equal(got, ref) and found is None:
            bad = int((got != ref).sum())
            found = f"mismatch: {'one' if mode == 1 else 'two'}-shot differs from the process group in {bad} of {n}"
    return found


def establish(group, ctrl, make, device, fault: Optional[str] = None):
    """Bring up a custom all-reduce for `group`, or agree to fall back to the process group.

    ``make(fault)`` constructs it (``XGMIAllReduce``; a stand-in in CPU tests) and must return an
    object with ``error`` set on any failure of this rank.  The ranks agree over `ctrl` (a CPU
    group: it still works when the device path is broken) first on construction, then on a
    ``cross_check`` against ``dist.all_reduce``.  Returns ``(custom or None, status)`` with status
    ``"on"`` or ``"fallback:<reason>"`` -- identical on every rank of the group."""
    import torch.distributed as dist

    def agree(reason):
        reasons = [None] * dist.get_world_size(ctrl)
        dist.all_gather_object(reasons, reason, group=ctrl)
        return next((f"rank{r}:{x}" for r, x in enumerate(reasons) if x), None)

    custom, reason = None, None
    try:
        custom = make(fault)
        reason = getattr(custom, "error", None)
    except Exception as exc:  # noqa: BLE001 -- a rank that cannot even construct still agrees
        reason = f"init: {exc}"
    reason = agree(reason)
    if reason is None:
        try:
            local = cross_check(custom, group, device, fault)
        except Exception as exc:  # noqa: BLE001
            local = f"cross-check: {exc}"
        reason = agree(local)
    if reason is None:
        return custom, "on"
    if custom is not None and hasattr(custom, "close"):
        custom.close()
    return None, f"fallback:{reason}"


class LocalRanks:
    """`world` ranks inside ONE process (buffers on the current GPU): a test harness
    for the collective kernels on a one-GPU box -- each rank launches on its own stream."""

    def __init__(self, world: int, cap_bytes: int = 4 << 20, oneshot_max: int = ONESHOT_MAX,
                 timeout_s: float = 5.0):
        lib = _lib()
        bufs = [_alloc(lib, cap_bytes) for _ in range(world)]
        data, sig = [b[0] for b in bufs], [b[1] for b in bufs]
        self.lib, self._bufs = lib, bufs
        self.ranks = [_Rank(lib, r, world, data, sig, cap_bytes, oneshot_max, timeout_s) for r in range(world)]

    def close(self):
        torch.cuda.synchronize()
        for d, s in self._bufs:
            self.lib.bcg_ar_free(ctypes.c_void_p(d))
            self.lib.bcg_ar_free(ctypes.c_void_p(s))
        self._bufs = []
