"""Process-group layout: one process per GPU, TP groups of consecutive ranks, DP across groups.

The reference delegates tensor parallelism to vLLM's multiprocessing executor
(``bcg/vllm_agent.py:126-142``: ``tensor_parallel_size`` +
``distributed_executor_backend='mp'``) and has no data parallelism inside a
run (``bcg/main.py:1073`` ``run_simulation`` is the external sweep hook).
Here both are explicit:

* ranks ``[g*tp, (g+1)*tp)`` form TP group ``g`` (RCCL all-reduce over xGMI:
  consecutive ranks of one node are direct xGMI peers on an MI355X OAM board);
* the ``world // tp`` groups are data-parallel replicas that run independent
  simulation seeds and only meet for the final result reduction.

``torch.distributed`` with backend ``"nccl"`` is RCCL on ROCm; CPU tests use
``"gloo"`` with the same code path.
"""

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

from ..models.transformer import TPGroup


@dataclass(frozen=True)
class Layout:
    world: int
    rank: int
    local_rank: int
    tp: int

    @property
    def dp(self) -> int:
        return self.world // self.tp

    @property
    def tp_rank(self) -> int:
        return self.rank % self.tp

    @property
    def dp_rank(self) -> int:
        return self.rank // self.tp

    @property
    def is_group_leader(self) -> bool:
        return self.tp_rank == 0


_TP_GROUPS = {}
_TP_CTRL = {}
_DP_GROUPS = {}
_CUSTOM_AR = {}
_CUSTOM_STATUS = {}


def env_layout(tp: int = 1) -> Layout:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world % tp:
        raise ValueError(f"world size {world} not divisible by tensor_parallel_size {tp}")
    return Layout(world, rank, local, tp)


def init_distributed(backend: Optional[str] = None, timeout_s: float = 600.0) -> Layout:
    """Initialise the default process group from torchrun's env (idempotent).

    Backend: RCCL (``"nccl"``) when a GPU is visible, gloo otherwise.  The
    rendezvous address defaults to 127.0.0.1 (single node; the container
    hostname may not resolve).
    """
    lay = env_layout()
    if lay.world == 1 or dist.is_initialized():
        return lay
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver
    if backend is None:
        backend = "nccl" if torch.cuda.device_count() > 0 else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(lay.local_rank)
    dist.init_process_group(backend, rank=lay.rank, world_size=lay.world,
                            timeout=datetime.timedelta(seconds=timeout_s))
    return lay


def tensor_parallel_group(tp: int, custom_allreduce: bool = False, hidden: Optional[int] = None) -> TPGroup:
    """TPGroup of this rank (every rank must call this with the same arguments).

    ``custom_allreduce``: also map the TP peers' buffers for the xGMI one-/two-shot
    all-reduce kernels (RCCL process groups on GPUs only; set
    ``BCG_CUSTOM_AR=0`` to force RCCL for every collective).  ``hidden``: the model's
    hidden size -- the calibration also times the fused all-reduce + add + RMSNorm
    kernels on rows of that width and routes them by their own one-shot limit.
    """
    if tp <= 1:
        return TPGroup()
    if not dist.is_initialized():
        init_distributed()
    lay = env_layout(tp)
    if dist.get_world_size() != lay.world:
        lay = Layout(dist.get_world_size(), dist.get_rank(), lay.local_rank, tp)
    if tp not in _TP_GROUPS:
        mine = ctrl = None
        gloo = dist.get_backend() == "gloo"
        for g in range(lay.world // tp):  # new_group is collective over ALL ranks
            ranks = list(range(g * tp, (g + 1) * tp))
            pg = dist.new_group(ranks)
            # the driver's scheduling plans travel over CPU: never queued on a HIP stream
            cg = pg if gloo else dist.new_group(ranks, backend="gloo")
            if lay.rank in ranks:
                mine, ctrl = pg, cg
        _TP_GROUPS[tp] = mine
        _TP_CTRL[tp] = ctrl
    mode = os.environ.get("BCG_CUSTOM_AR", "1")  # 0 = RCCL only, force = also over gloo (1-GPU tests)
    if custom_allreduce and mode != "0" and (mode == "force" or dist.get_backend(_TP_GROUPS[tp]) == "nccl"):
        if tp not in _CUSTOM_STATUS:
            _CUSTOM_AR[tp], _CUSTOM_STATUS[tp] = _establish_custom(tp, hidden)
    else:
        _CUSTOM_STATUS.setdefault(tp, "off")
    g = TPGroup(_TP_GROUPS[tp], lay.tp_rank, tp, custom=_CUSTOM_AR.get(tp), ctrl=_TP_CTRL[tp],
                leader=lay.rank - lay.tp_rank, chunk_large=dist.get_backend(_TP_GROUPS[tp]) == "gloo")
    g.custom_status = _CUSTOM_STATUS[tp]
    return g


def _establish_custom(tp: int, hidden: Optional[int]):
    """The xGMI all-reduce of this rank's TP group, cross-checked against the process group, or
    an agreed fallback to it (``custom_allreduce.establish``): a first run on a node whose IPC
    mapping or peer access fails serves through RCCL instead of dying at TP init.
    ``BCG_AR_FAULT=ipc|mismatch`` injects either failure (tests)."""
    from .custom_allreduce import XGMIAllReduce, establish
    group, ctrl = _TP_GROUPS[tp], _TP_CTRL[tp]
    fault = os.environ.get("BCG_AR_FAULT") or None
    # BCG_AR_CAP_MB: largest message of the xGMI kernels (RCCL above it; over gloo the larger
    # messages go through the kernels in cap-sized pieces, TPGroup.chunk_large)
    make = lambda f: XGMIAllReduce(group, cap_bytes=int(os.environ.get("BCG_AR_CAP_MB", "32")) << 20,  # noqa: E731
                                   timeout_s=float(os.environ.get("BCG_AR_TIMEOUT_S", "30")), fault=f)
    custom, status = establish(group, ctrl, make, torch.device("cuda", torch.cuda.current_device()), fault)
    if custom is None:
        return None, status
    # routing limits measured on this group's links (RCCL groups; BCG_AR_CALIBRATE=0 keeps the
    # built-in rule, =force also calibrates over gloo -- one-GPU tests of the mechanism)
    cal = os.environ.get("BCG_AR_CALIBRATE", "1")
    if cal == "force" or (cal != "0" and dist.get_backend(group) == "nccl"):
        custom.calibrate(group, route=dist.get_backend(group) == "nccl", hidden=hidden)
    return custom, status


def data_parallel_group(tp: int):
    """Group of the TP-rank-0 processes (one per replica) for result reduction; None if world == tp."""
    if not dist.is_initialized():
        return None
    world = dist.get_world_size()
    if world == tp:
        return None
    if tp not in _DP_GROUPS:
        _DP_GROUPS[tp] = dist.new_group(list(range(0, world, tp)))
    return _DP_GROUPS[tp]


def destroy():
    for ar in _CUSTOM_AR.values():
        if ar is not None:
            ar.close()
    _CUSTOM_AR.clear()
    _CUSTOM_STATUS.clear()
    _TP_GROUPS.clear()
    _TP_CTRL.clear()
    _DP_GROUPS.clear()
    if dist.is_initialized():
        dist.destroy_process_group()
