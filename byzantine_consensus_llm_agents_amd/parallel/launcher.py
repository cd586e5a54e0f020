"""Self-launch of tensor-parallel worker processes (the vLLM ``mp`` executor's role).

The reference gets its TP workers from vLLM: ``LLM(**llm_args)`` with
``tensor_parallel_size=N`` and ``distributed_executor_backend='mp'``
(``bcg/vllm_agent.py:126-144``) -- a plain ``python main.py`` run.  Here
``LLM(..., tensor_parallel_size=N)`` in a process that no launcher started
(no ``WORLD_SIZE``) calls :func:`spawn_tp_workers`:

* ranks 1..N-1 are started as child processes running
  ``python -m byzantine_consensus_llm_agents_amd.engine.tp_worker`` with the
  same engine arguments and ``ENGINE_CONFIG`` (JSON in ``BCG_TP_WORKER_SPEC``);
* this process becomes rank 0 (the driver) of a 127.0.0.1 rendezvous;
* everything happens BEFORE this process touches the GPU (a process that
  initialised HIP must not fork/exec children on this platform).

Under torchrun (``WORLD_SIZE`` set) nothing is spawned: every rank builds the
engine itself and the followers call ``LLM.serve_worker()``.
"""

import json
import os
import socket
import subprocess
import sys
import time
from typing import Dict, List, Optional

WORKER_MODULE = "byzantine_consensus_llm_agents_amd.engine.tp_worker"


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class Workers:
    """The spawned follower processes of one TP group."""

    def __init__(self, procs: List[subprocess.Popen]):
        self.procs = procs

    def alive(self) -> bool:
        return all(p.poll() is None for p in self.procs)

    def join(self, timeout: float = 120.0) -> List[Optional[int]]:
        """Wait for the followers (they exit when the driver's engine sends stop)."""
        deadline = time.monotonic() + timeout
        codes = []
        for p in self.procs:
            try:
                codes.append(p.wait(timeout=max(0.1, deadline - time.monotonic())))
            except subprocess.TimeoutExpired:
                p.kill()  # our own child, by PID
                codes.append(p.wait())
        return codes


def spawn_tp_workers(tp: int, llm_kwargs: Dict) -> Optional[Workers]:
    """Spawn ranks 1..tp-1 and make this process rank 0, unless a launcher already did."""
    if tp <= 1 or os.environ.get("WORLD_SIZE"):
        return None
    import torch
    if torch.cuda.is_initialized():
        raise RuntimeError("tensor_parallel_size > 1: the TP workers must be spawned before this process "
                           "uses the GPU (create the LLM first, or launch with torchrun)")
    from ..bcg.config import ENGINE_CONFIG
    port = _free_port()
    base = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(tp),
                HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    spec = {"llm": llm_kwargs, "engine_config": {k: v for k, v in ENGINE_CONFIG.items()
                                                 if isinstance(v, (str, int, float, bool, type(None)))}}
    base["BCG_TP_WORKER_SPEC"] = json.dumps(spec)
    root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    base["PYTHONPATH"] = root + (os.pathsep + base["PYTHONPATH"] if base.get("PYTHONPATH") else "")
    procs = []
    for r in range(1, tp):
        env = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, "-m", WORKER_MODULE], env=env, cwd=root))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(tp), RANK="0",
                      LOCAL_RANK="0")
    return Workers(procs)
