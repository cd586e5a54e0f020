"""User-facing engine API (the L0 boundary the reference reached through vLLM).

``LLM.generate(prompts, sampling_params)`` mirrors the vLLM call sites used by
the reference (``bcg/vllm_agent.py:144, :331, :430``) with one extension that
removes the reference's batch-size-1 fallback: ``sampling_params`` may be a
*list*, one per prompt, each with its own ``GuidedDecodingParams(json=...)``.

Backends:
  * ``hip``   - :class:`..engine.engine.InferenceEngine` with the HIP kernels
                (MI355X); fails loudly if the kernel library is missing;
  * ``torch`` - the same engine on PyTorch reference ops (CPU tests);
  * ``fake``  - scripted schema-valid answers (plumbing, parity tests);
  * ``hostmodel`` - the engine's host work (tokenize, detokenize) with a modelled GPU at a
                measured token rate (host-budget measurements of several DP ranks).

Tensor parallelism: ``tensor_parallel_size > 1`` in a process that was not
started by a launcher spawns the TP worker processes itself (ranks 1..N-1, each
running :mod:`.tp_worker`), like vLLM's ``mp`` executor; this process becomes
the group's driver.  Under an external launcher (torchrun) every rank builds
the same ``LLM``; ``is_driver`` tells the group's rank 0 (serves requests) from
the followers (``serve_worker`` / ``start_worker``).

Several simulations may share one ``LLM`` from different threads.  With
``start_continuous_batching()`` every call's sequences join the
engine's running decode batch as soon as they arrive and leave it when they
finish (iteration-level scheduling).  Otherwise calls are coalesced
(:class:`Coalescer`) into one batch once every registered thread waits on the
engine -- deterministic batch composition, required when TP ranks must make
identical scheduling decisions.
"""

import os
import threading
import time
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Sequence, Union

from ..bcg.config import ENGINE_CONFIG


@dataclass
class GuidedDecodingParams:
    json: Optional[Dict[str, Any]] = None


@dataclass
class SamplingParams:
    temperature: float = 1.0
    top_p: float = 1.0
    max_tokens: int = 16
    guided_decoding: Optional[GuidedDecodingParams] = None
    seed: Optional[int] = None


@dataclass
class CompletionOutput:
    index: int
    text: str
    token_ids: List[int] = field(default_factory=list)
    finish_reason: str = "stop"


@dataclass
class RequestOutput:
    request_id: int
    prompt: str
    outputs: List[CompletionOutput]
    num_prompt_tokens: int = 0
    num_cached_tokens: int = 0


class Coalescer:
    """Merge concurrent ``generate`` calls from registered threads into one batch."""

    def __init__(self, run_batch):
        self._run = run_batch
        self._cond = threading.Condition()
        self._participants = 0
        self._tickets: List[dict] = []

    def join(self):
        with self._cond:
            self._participants += 1

    def leave(self):
        with self._cond:
            self._participants -= 1
            self._maybe_flush_locked()

    def _maybe_flush_locked(self):
        waiting = [t for t in self._tickets if not t["done"]]
        if waiting and len(waiting) >= self._participants:
            self._tickets = []
            self._cond.release()
            try:
                self._flush(waiting)
            finally:
                self._cond.acquire()
            self._cond.notify_all()

    def _flush(self, tickets):
        # deterministic row order (TP ranks must build identical batches)
        tickets = sorted(tickets, key=lambda t: t["key"])
        prompts, params, spans = [], [], []
        for t in tickets:
            spans.append((len(prompts), len(t["prompts"])))
            prompts += t["prompts"]
            params += t["params"]
        try:
            texts = self._run(prompts, params)
            for t, (a, n) in zip(tickets, spans):
                t["result"] = texts[a:a + n]
        except Exception as exc:  # every caller sees the engine failure
            for t in tickets:
                t["error"] = exc
        for t in tickets:
            t["done"] = True

    def submit(self, prompts, params):
        key = getattr(threading.current_thread(), "_bcg_order_key", ())
        ticket = {"prompts": prompts, "params": params, "done": False, "key": key}
        with self._cond:
            self._tickets.append(ticket)
            self._maybe_flush_locked()
            while not ticket["done"]:
                self._cond.wait()
        if "error" in ticket:
            raise ticket["error"]
        return ticket["result"]


def resolve_backend(requested: Optional[str]) -> str:
    name = (requested or ENGINE_CONFIG.get("backend") or "auto").lower()
    if name != "auto":
        return name
    try:
        import torch
        if torch.cuda.device_count() > 0:
            return "hip"
    except Exception:
        pass
    return "fake"


class LLM:
    """In-process engine facade (one per process / TP group)."""

    def __init__(self, model: str, max_model_len: int = 8192, gpu_memory_utilization: float = 0.9,
                 tensor_parallel_size: int = 1, max_num_seqs: Optional[int] = None,
                 quantization: Optional[str] = None, backend: Optional[str] = None,
                 weights: Optional[str] = None, seed: Optional[int] = None, **kwargs):
        self.model = model
        self.backend_name = resolve_backend(backend)
        seed = seed if seed is not None else ENGINE_CONFIG.get("seed")
        self.workers = None
        if self.backend_name == "fake":
            from .fake import FakeBackend
            self.backend = FakeBackend(seed=seed or 0)
            # scripted engine: no model to shard; under a TP layout only each group's rank 0 serves
            self.backend.is_driver = int(os.environ.get("RANK", "0")) % max(1, tensor_parallel_size) == 0
        elif self.backend_name == "hostmodel":
            # host work of the real engine + a modelled GPU (host-budget measurements, bench.py)
            from .fake import HostModelBackend
            self.backend = HostModelBackend(model, seed=seed or 0,
                                            tokens_per_s=float(os.environ.get("BCG_HOSTMODEL_TOKENS_S", "34000")))
            self.backend.is_driver = int(os.environ.get("RANK", "0")) % max(1, tensor_parallel_size) == 0
        elif self.backend_name in ("hip", "torch"):
            if tensor_parallel_size > 1:
                # the reference's entry point gets TP workers from vLLM's 'mp' executor
                # (bcg/vllm_agent.py:139-142); here: spawn them unless a launcher did
                from ..parallel.launcher import spawn_tp_workers
                self.workers = spawn_tp_workers(tensor_parallel_size, dict(
                    model=model, max_model_len=max_model_len, gpu_memory_utilization=gpu_memory_utilization,
                    tensor_parallel_size=tensor_parallel_size, max_num_seqs=max_num_seqs,
                    quantization=quantization, backend=self.backend_name, weights=weights, seed=seed,
                    **kwargs))
            from .engine import EngineArgs, InferenceEngine
            args = EngineArgs.from_configs(model, max_model_len=max_model_len,
                                           gpu_memory_utilization=gpu_memory_utilization,
                                           tensor_parallel_size=tensor_parallel_size,
                                           max_num_seqs=max_num_seqs, quantization=quantization,
                                           backend=self.backend_name, weights=weights, seed=seed,
                                           **kwargs)
            self.backend = InferenceEngine(args)
        else:
            raise ValueError(f"unknown engine backend {self.backend_name!r}")
        # every call goes through the coalescer: with no registered clients it
        # flushes immediately, with N registered threads it waits for all of them
        self.coalescer = Coalescer(self._run_batch)
        self._next_id = 0
        self.stats = {"calls": 0, "sequences": 0, "seconds": 0.0}

    # --------------------------------------------------- multi-sim sharing
    def register_client(self):
        """Declare one more thread whose calls should be coalesced with the others'."""
        self.coalescer.join()

    def unregister_client(self):
        self.coalescer.leave()

    # ------------------------------------------------------------- serving
    def _run_batch(self, prompts: List[str], params: List[SamplingParams]) -> List[str]:
        t0 = time.perf_counter()
        texts = self.backend.generate(prompts, params)
        self.stats["calls"] += 1
        self.stats["sequences"] += len(prompts)
        self.stats["seconds"] += time.perf_counter() - t0
        return texts

    def generate(self, prompts: Union[str, Sequence[str]],
                 sampling_params: Union[SamplingParams, Sequence[SamplingParams], None] = None,
                 use_tqdm: bool = False) -> List[RequestOutput]:
        if isinstance(prompts, str):
            prompts = [prompts]
        prompts = list(prompts)
        if sampling_params is None:
            sampling_params = SamplingParams()
        if isinstance(sampling_params, SamplingParams):
            params = [sampling_params] * len(prompts)
        else:
            params = list(sampling_params)
            if len(params) != len(prompts):
                raise ValueError("need one SamplingParams per prompt")
        if not prompts:
            return []
        if getattr(self.backend, "async_mode", False):
            # continuous batching: requests join the running batch directly
            texts = self._run_batch(prompts, params)
        else:
            texts = self.coalescer.submit(prompts, params)
        outs = []
        for p, t in zip(prompts, texts):
            outs.append(RequestOutput(self._next_id, p, [CompletionOutput(0, t)]))
            self._next_id += 1
        return outs

    @property
    def is_driver(self) -> bool:
        """False on a TP follower rank (it serves no requests, it replays the driver's plans)."""
        return getattr(self.backend, "is_driver", True)

    def start_continuous_batching(self):
        """Switch the engine to its background scheduler (iteration-level batching; TP drivers too)."""
        if hasattr(self.backend, "start_async"):
            self.backend.start_async()

    def start_worker(self):
        """TP follower: replay the driver's plans on a background thread until it stops."""
        if hasattr(self.backend, "start_follower"):
            self.backend.start_follower()

    def serve_worker(self):
        """TP follower: replay the driver's plans on this thread until it stops (blocking)."""
        if hasattr(self.backend, "serve_follower"):
            self.backend.serve_follower()

    def precompile(self, schemas):
        """Compile JSON-schema FSMs up front (no-op for the scripted backend)."""
        if hasattr(self.backend, "precompile"):
            self.backend.precompile(schemas)

    def shutdown(self):
        self.backend.shutdown()
        if self.workers is not None:
            self.workers.join()
            self.workers = None
