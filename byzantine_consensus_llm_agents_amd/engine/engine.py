"""The in-process inference engine: one batched prefill + device-driven decode per call.

``InferenceEngine.generate(prompts, params)`` is what every BCG phase calls
(through ``LLM.generate``).  For one call:

1. tokenise all prompts (HF ``tokenizers``, Rust, batched);
2. admit sequences into the paged KV pool (native ``BlockManager``); full
   prompt blocks that an earlier call already computed -- the agent's system
   prompt and chat header, identical every round -- are reused and skipped;
3. prefill every sequence's uncached suffix in packed chunks (varlen
   attention over paged KV) and sample each first token;
4. decode all sequences together: each step is embedding -> L layers ->
   LM head -> fused FSM-mask + Gumbel sampling, entirely on the device (the
   HIP backend replays a captured HIP graph per batch bucket); the host only
   polls the ``done`` flags every few steps;
5. detokenise, release blocks (prompt blocks stay cached).

Heterogeneous JSON schemas, temperatures and max_tokens coexist in one batch:
they are per-row device state (``fsm_base/fsm_state``, ``temperature``,
``max_new``).

Threads.  ``submit`` (any caller thread) only does CPU work -- tokenise,
compile the schema's token FSM -- and appends to ``_incoming``.  Everything
that touches the device or the schedule runs on ONE scheduler thread (the
background thread in async mode): each iteration first drains ``_incoming``
into the admission queue and installs new FSM tables, so the admission order
and the FSM row bases are decided in one place.

Tensor parallelism (driver / follower).  In a TP group only rank 0 (the
driver) owns requests and makes scheduling decisions; the other ranks are
followers that hold their weight shards and replay the driver's schedule.
Every iteration the driver broadcasts a small plan over a CPU (gloo) group --
the requests it drained this iteration (token ids, limits, schema) and the one
timing-dependent decision (launch the next burst before reaping) -- and each
follower applies it to its own identical engine state.  Everything else
(admission, KV blocks, compaction, buckets, sampling) is a deterministic
function of that plan sequence and of device data that is bitwise identical on
every rank (identical all-reduce / all-gather results, counter-based sampling),
so all ranks launch the same forwards and collectives in the same order while
the driver keeps iteration-level continuous batching (the vLLM ``mp``
executor's model: ``bcg/vllm_agent.py:139-142``).
"""

import collections
import contextlib
import json
import os
import threading
import time
from dataclasses import dataclass, field
from typing import Deque, Dict, List, Optional

import numpy as np
import torch

from ..bcg.config import ENGINE_CONFIG
from ..models.config import ModelConfig, get_model_config
from ..models.transformer import AttnMeta, DecoderModel, TPGroup
from ..ops import get_ops
from ..utils.trace import PhaseTimer
from .guided.compiler import FSMRegistry
from .tokenizer import load_tokenizer

OUT_WIDTH = 1024  # max generated tokens per sequence (the reference uses <= 300)


@dataclass
class EngineArgs:
    model: str
    model_cfg: ModelConfig
    backend: str = "hip"
    weights: str = "random"
    seed: Optional[int] = None
    max_model_len: int = 8192
    tensor_parallel_size: int = 1
    gpu_memory_utilization: float = 0.9
    max_num_seqs: Optional[int] = None
    quantization: Optional[str] = None
    kv_block_size: int = 16
    max_batch_seqs: int = 512
    prefill_chunk_tokens: int = 16384
    budget_aware_json: bool = False
    # benchmark grammar for untrained weights: every property emitted, free-text strings with
    # >= this many visible characters (guided/json_schema.py validity_aware); 0 = the schema as given
    validity_aware_json: int = 0
    # ... and its free text printable ASCII (late-game prompts stay in the reference's bounded sizes)
    ascii_text_json: bool = False
    max_whitespace: int = 4
    prefix_caching: bool = True
    use_hip_graphs: bool = True
    kv_cache_gb: Optional[float] = None
    honor_max_num_seqs: bool = False
    dtype: torch.dtype = torch.bfloat16
    device: Optional[str] = None
    poll_every: int = 8
    async_mode: bool = False
    precapture_graphs: bool = True  # capture every decode bucket at the first burst (and after FSM growth)
    kv_cache_dtype: str = "auto"    # "auto" = activation dtype (bf16); "fp8" = OCP e4m3fn (half the KV bytes)
    # admission batching (0 = admit at once): queue prompts for up to this many decode
    # bursts while >= admit_min_live rows decode, until >= frac x prefill_chunk_tokens wait
    admit_max_wait: int = 0
    admit_min_live: int = 64
    admit_min_tokens_frac: float = 1.5
    # full prefill chunks only while the decode batch is fed: the last, partial chunk of a wave
    # is carried (its prompts stay pending with their KV so far) into the next wave, for at most
    # this many more bursts; 0 = every wave runs its tail chunk at once
    prefill_carry_bursts: int = 0
    # decode attention reads KV blocks shared by several rows (prefix cache) once per group
    # of rows instead of once per row (engine/cascade.py); HIP backend only
    cascade_decode: bool = True

    @classmethod
    def from_configs(cls, model: str, backend: str, weights: Optional[str] = None,
                     seed: Optional[int] = None, **kw) -> "EngineArgs":
        ec = ENGINE_CONFIG
        weights = weights or ec.get("weights") or "auto"
        model_dir = weights if weights not in ("auto", "random") else None
        cfg = get_model_config(model, model_dir)
        if ec.get("num_layers_override"):
            # reduced depth at the real layer shapes: end-to-end tests of large configurations
            # (TP engines on a one-GPU box) -- never a measurement (bench.py refuses it)
            import dataclasses
            cfg = dataclasses.replace(cfg, num_layers=int(ec["num_layers_override"]))
        args = cls(model=model, model_cfg=cfg, backend=backend,
                   weights="random" if weights == "auto" else weights, seed=seed,
                   kv_block_size=ec.get("kv_block_size", 16),
                   max_batch_seqs=ec.get("max_batch_seqs", 512),
                   prefill_chunk_tokens=ec.get("prefill_chunk_tokens", 16384),
                   budget_aware_json=ec.get("budget_aware_json", False),
                   validity_aware_json=int(ec.get("validity_aware_json", 0)),
                   ascii_text_json=bool(ec.get("ascii_text_json", False)),
                   max_whitespace=ec.get("max_whitespace", 4),
                   prefix_caching=ec.get("prefix_caching", True),
                   use_hip_graphs=ec.get("use_hip_graphs", True),
                   kv_cache_gb=ec.get("kv_cache_gb"),
                   honor_max_num_seqs=ec.get("honor_max_num_seqs", False),
                   precapture_graphs=ec.get("precapture_graphs", True),
                   kv_cache_dtype=ec.get("kv_cache_dtype", "auto"),
                   admit_max_wait=int(ec.get("admit_max_wait", 0)),
                   poll_every=max(1, int(ec.get("poll_every", 8))),
                   prefill_carry_bursts=int(ec.get("prefill_carry_bursts", 0)),
                   cascade_decode=bool(ec.get("cascade_decode", True)))
        dtype = ec.get("dtype", "bfloat16")
        args.dtype = getattr(torch, dtype) if isinstance(dtype, str) else dtype
        for key, value in kw.items():
            if value is not None and hasattr(args, key):
                setattr(args, key, value)
        return args


@dataclass
class _Seq:
    idx: int
    prompt_ids: List[int]
    max_new: int
    temperature: float
    fsm_key: Optional[str]          # compiled schema key (None = unguided)
    fsm_base: int = -1              # device row base, assigned by the scheduler thread
    blocks: List[int] = field(default_factory=list)
    cached: int = 0
    done_pos: int = 0               # prompt tokens whose KV is written (prefix cache + prefilled chunks)
    error: Optional[str] = None
    max_new_requested: int = 0      # the caller's max_tokens (before the context-room clamp)


class InferenceEngine:
    def __init__(self, args: EngineArgs):
        self.args = args
        self.timer = PhaseTimer()
        self.stats = {"prompt_tokens": 0, "cached_tokens": 0, "generated_tokens": 0,
                      "decode_steps": 0, "decode_row_steps": 0, "prefill_chunks": 0, "prefill_full_chunks": 0,
                      "prefill_tail_tokens": 0, "prefill_carried": 0, "calls": 0,
                      # prompts with no room for one token (n >= max_model_len): answered "" at once
                      "context_rejects": 0,
                      # prompts whose context room cut max_tokens below the grammar's shortest
                      # complete output (the answer cannot be valid JSON)
                      "context_short": 0,
                      # prompts holding lone UTF-16 surrogates (tokenised with U+FFFD in their place)
                      "prompts_sanitized": 0}
        # prompt token counts per requested max_tokens (bench.py: decide 300 / vote 200), in
        # submission order: callers slice them by position for a time window's percentiles
        self.prompt_lens: Dict[int, List[int]] = collections.defaultdict(list)
        self._carry: List["_Request"] = []  # admitted, prefill incomplete (pending), oldest first
        cfg = args.model_cfg
        self.backend = args.backend
        if self.backend == "hip" and not torch.cuda.is_available():
            raise RuntimeError("hip backend requested but no GPU is visible")
        # TP first: joining the process group selects this rank's GPU (LOCAL_RANK)
        self.tp = self._init_tp(args.tensor_parallel_size, cfg.hidden_size)
        if args.device:
            self.device = torch.device(args.device)
        elif self.backend == "hip":
            self.device = torch.device("cuda", torch.cuda.current_device())
        else:
            self.device = torch.device("cpu")
        self.ops = get_ops(self.backend)

        model_dir = args.weights if args.weights not in ("random", "auto") else None
        self.tokenizer = load_tokenizer(args.model, model_dir)
        if self.tokenizer.vocab_size > cfg.vocab_size:
            raise ValueError("tokenizer larger than the model vocabulary")
        self.model = DecoderModel(cfg, self.ops, self.device, args.dtype, self.tp, quant=args.quantization)
        with self.timer.phase("load_weights"):
            if model_dir:
                from ..models.loader import load_safetensors_dir
                self.model.load_hf_state_dict(load_safetensors_dir(model_dir))
            else:
                self.model.init_random(seed=args.seed or 0)
        self.seed = (args.seed if args.seed is not None else int.from_bytes(os.urandom(4), "little")) & 0x7FFFFFFF
        if self.tp.size > 1:  # TP ranks sample identically: share rank 0's seed
            t = torch.tensor([self.seed], dtype=torch.int64,
                             device=self.device if self.device.type == "cuda" else "cpu")
            torch.distributed.broadcast(t, src=torch.distributed.get_global_rank(self.tp.group, 0),
                                        group=self.tp.group)
            self.seed = int(t.item())
        self._req_counter = 0

        self.fsm = FSMRegistry(self.tokenizer.all_token_bytes(), cfg.vocab_size, self.device,
                               max_ws=args.max_whitespace, validity_aware_min=args.validity_aware_json,
                               ascii_text=args.ascii_text_json)
        self.eos_ids = (self.tokenizer.eos_token_ids + [self.tokenizer.eos_token_ids[0]])[:2]
        self.n_text_tokens = min(self.tokenizer.vocab_size, cfg.vocab_size)
        self._alloc_kv_cache()
        if self.backend == "hip":
            self._load_tuned_gemms()
        self._alloc_state()
        self._cv = threading.Condition()
        self._incoming: List[_Request] = []        # submitted, not yet seen by the scheduler
        self._waiting: Deque[_Request] = collections.deque()  # admission queue (scheduler thread)
        self.is_driver = self.tp.rank == 0
        self.async_mode = False
        self._follower = None
        self._fatal: Optional[BaseException] = None
        self._stop = False
        self._ar_err_host = None
        self.graphs = None
        # Prefill runs on the engine's one stream between decode bursts.  (A second prefill
        # stream concurrent with the bursts lost three A/Bs, the last -2.9 % tokens/s: every
        # 256x256 GEMM holds a CU's whole LDS, so the two streams only time-share the CUs --
        # PERF.md "Overlapped prefill"; removed in round 5.)
        if hasattr(self.ops, "prepare_device"):  # split-K counters: allocated before any graph capture
            self.ops.prepare_device(self.device)
        self._skip_done_attn = os.environ.get("BCG_SKIP_DONE_ATTN", "1") != "0"
        self._bursts = 0         # decode bursts launched (admission-batching clock)
        self._snap = None        # host copy of (done, gen_count, out_tokens) after the last burst
        self._engine_errors = 0
        self._snap_buf = None
        # under TP without the xGMI kernels (not requested, or an agreed fallback at init) every
        # decode collective is a process-group call: decode runs eagerly -- a collective of the
        # process group inside a captured HIP graph is a path this build does not test
        # (BCG_TP_GRAPHS_WITH_PG=1 captures anyway)
        self.graphs_off_reason = None
        if (self.backend == "hip" and args.use_hip_graphs and self.tp.size > 1 and self.tp.custom is None
                and os.environ.get("BCG_TP_GRAPHS_WITH_PG") != "1"):
            self.graphs_off_reason = f"tp collectives through the process group ({self.tp.custom_status})"
        if self.backend == "hip" and args.use_hip_graphs and self.graphs_off_reason is None:
            from .graphs import DecodeGraphs
            self.graphs = DecodeGraphs(self)

    # ------------------------------------------------------------- setup
    def _init_tp(self, tp_size: int, hidden: int) -> TPGroup:
        if tp_size <= 1:
            return TPGroup()
        from ..parallel.groups import tensor_parallel_group
        return tensor_parallel_group(tp_size, custom_allreduce=(
            self.backend == "hip" and ENGINE_CONFIG.get("custom_allreduce", True)), hidden=hidden)

    def kv_dtype(self) -> torch.dtype:
        kd = (self.args.kv_cache_dtype or "auto").lower()
        if kd == "auto":
            return self.args.dtype
        if kd in ("fp8", "fp8_e4m3", "float8_e4m3fn"):
            return torch.float8_e4m3fn
        raise ValueError(f"unsupported kv_cache_dtype {self.args.kv_cache_dtype!r} (auto | fp8)")

    def _alloc_kv_cache(self):
        a, m = self.args, self.model
        bs = a.kv_block_size
        kv_dtype = self.kv_dtype()
        per_block = 2 * m.cfg.num_layers * m.n_kv * bs * m.hd * torch.tensor([], dtype=kv_dtype).element_size()
        want_tokens = a.max_batch_seqs * a.max_model_len
        if a.kv_cache_gb:
            budget = int(a.kv_cache_gb * 2 ** 30)
        elif self.device.type == "cuda":
            free, total = torch.cuda.mem_get_info(self.device)
            # prefill activations of one chunk + the decode graphs' private pool (largest
            # bucket: logits / sampler temporaries, MLP activations) + the shared split-K scratch
            from .graphs import MAX_ROWS
            rows = min(a.max_batch_seqs, MAX_ROWS)
            graphs = rows * (m.cfg.vocab_size * 8 + 8 * m.inter + 16 * m.cfg.hidden_size) * 2
            reserve = (6 * 2 ** 30 + 2 * a.prefill_chunk_tokens * (m.cfg.hidden_size + 2 * m.inter) * 2
                       + graphs + self._decode_ws_bytes())
            budget = int(min(free - reserve, total * a.gpu_memory_utilization - torch.cuda.memory_allocated(self.device)))
        else:
            budget = 256 * 2 ** 20
        num_blocks = max(16, min(budget // per_block, want_tokens // bs + 1))
        self.k_cache = torch.zeros((m.cfg.num_layers, num_blocks, m.n_kv, bs, m.hd), dtype=kv_dtype,
                                   device=self.device)
        # V is stored transposed per block-head (see ops/reference.py)
        self.v_cache = torch.zeros((m.cfg.num_layers, num_blocks, m.n_kv, m.hd, bs), dtype=kv_dtype,
                                   device=self.device)
        from ..runtime import BlockManager
        # block 0 is scratch (padding rows of graph buckets write there); never handed out
        self.blocks = BlockManager(num_blocks - 1, bs)
        self.num_blocks = num_blocks
        self.max_blocks_per_seq = (a.max_model_len + bs - 1) // bs
        self.kv_bytes = 2 * self.k_cache.numel() * self.k_cache.element_size()

    def _decode_ws_bytes(self) -> int:
        if not hasattr(self.ops, "decode_workspace_numel"):
            return 0
        from .graphs import MAX_ROWS
        a, m = self.args, self.model
        rows = min(MAX_ROWS, max(a.max_batch_seqs, 1))
        max_blocks = (a.max_model_len + a.kv_block_size - 1) // a.kv_block_size
        cascade = bool(a.cascade_decode)
        limit = self.ops.decode_max_context(cascade)
        if max_blocks * a.kv_block_size > limit:  # fail at init, not with rc -3 at the first decode
            raise ValueError(f"max_model_len {a.max_model_len} exceeds the decode attention limit of {limit} "
                             f"tokens ({'with' if cascade else 'without'} shared-prefix decode; "
                             "cascade_decode=False allows 16384)")
        return 4 * self.ops.decode_workspace_numel(rows, m.n_q, m.hd, max_blocks, a.kv_block_size, cascade)

    def _load_tuned_gemms(self):
        """Load PyTorch TunableOp results for this model's decode GEMM shapes (lookups only).

        ``tools/tune_gemms.py`` times every hipBLASLt/rocBLAS solution per decode
        bucket; e.g. Qwen3-14B down_proj at M=160 goes 126 -> 54 us.  Unknown
        shapes (prefill) fall back to the library default, no tuning at run time.
        """
        if os.environ.get("BCG_TUNABLEOP", "1") == "0":
            return
        name = self.args.model.split("/")[-1].lower()
        path = os.path.join(os.path.dirname(__file__), "tuned",
                            f"tunableop_{name}_tp{self.args.tensor_parallel_size}.csv")
        if not os.path.exists(path):
            return
        import tempfile
        t = torch.cuda.tunable
        t.enable(True)
        t.tuning_enable(False)
        t.set_filename(os.path.join(tempfile.gettempdir(), f"bcg_tunableop_{os.getpid()}.csv"))
        t.read_file(path)
        self.tuned_gemm_file = path

    def _alloc_state(self):
        """Per-row decode state, shared by every graph bucket (bucket b uses rows [0, b))."""
        from .graphs import MAX_ROWS
        cap = min(MAX_ROWS, max(self.args.max_batch_seqs, 1))
        dev = self.device
        z = lambda: torch.zeros(cap, dtype=torch.int32, device=dev)  # noqa: E731
        self.state = {
            "block_tables": torch.zeros(cap, self.max_blocks_per_seq, dtype=torch.int32, device=dev),
            "seq_lens": torch.ones(cap, dtype=torch.int32, device=dev),
            "fsm_base": torch.full((cap,), -1, dtype=torch.int32, device=dev),
            "fsm_state": z(), "gen_count": z(), "max_new": torch.ones(cap, dtype=torch.int32, device=dev),
            "temperature": torch.zeros(cap, dtype=torch.float32, device=dev), "row_keys": z(),
            "done": torch.ones(cap, dtype=torch.int32, device=dev), "next_tokens": z(),
            "out_tokens": torch.zeros(cap, OUT_WIDTH, dtype=torch.int32, device=dev)}
        self.slots: List[Optional[_Request]] = [None] * cap
        # one split-K scratch for every decode graph (they never run concurrently); every
        # partial is written before it is read, so no initialisation is needed
        ws = self._decode_ws_bytes() // 4
        self.decode_ws = torch.empty(ws, dtype=torch.float32, device=dev) if ws else None
        self.cascade = None
        if self.backend == "hip" and self.args.cascade_decode and os.environ.get("BCG_CASCADE", "1") != "0":
            from .cascade import CascadeTables
            self.cascade = CascadeTables(cap, dev, self.args.kv_block_size)
        self._layout_dirty = True  # live rows changed since the cascade tables were built
        rows_fn = getattr(self.ops, "prefill_tile_rows", None)
        self._tile_rows = (rows_fn(self.model.hd, self.kv_dtype() == torch.float8_e4m3fn, self.max_blocks_per_seq)
                           if rows_fn else 64)

    def _phys(self, blocks: List[int]) -> List[int]:
        return [b + 1 for b in blocks]  # manager ids are shifted past scratch block 0

    # ------------------------------------------------------------ serving
    def generate(self, prompts: List[str], params_list) -> List[str]:
        """Serve one batch of prompts; returns the generated texts in order.

        Async mode (continuous batching): the requests join the running batch of
        the background scheduler thread and this call waits for them.  Sync
        mode: the calling thread drives the scheduler until they are done.
        """
        if not self.is_driver:
            raise RuntimeError("generate() on a TP follower: only the group's rank 0 serves requests")
        reqs = self.submit(prompts, params_list)
        if self.async_mode:
            for r in reqs:
                r.event.wait()
        else:
            with self._device_ctx():
                while not all(r.event.is_set() for r in reqs):
                    self._iterate()
        for r in reqs:
            if r.exc is not None:
                raise r.exc
        return [r.text for r in reqs]

    def _make_request(self, p_ids: List[int], max_tokens: int, temperature: float,
                      fsm_key: Optional[str]) -> "_Request":
        seq = _Seq(0, list(p_ids), max(1, int(max_tokens)), float(temperature), fsm_key,
                   max_new_requested=int(max_tokens))
        req = _Request(seq)
        n, limit = len(p_ids), self.args.max_model_len
        if n == 0 or n >= limit:
            req.limit = "context_rejects"
            req.finish("")  # no room for even one token: the caller sees an unparsable (empty) output
        else:
            # generate up to the context limit, as vLLM does (not an empty answer)
            seq.max_new = min(seq.max_new, limit - n, OUT_WIDTH)
            if fsm_key is not None and seq.max_new < int(max_tokens):
                shortest = int(self.fsm._fsms[fsm_key].dist[0]) if fsm_key in self.fsm._fsms else 0
                if seq.max_new < shortest:
                    req.limit = "context_short"
        return req

    def submit(self, prompts: List[str], params_list) -> List["_Request"]:
        """Tokenise + compile schemas on the caller's thread (CPU only), hand to the scheduler."""
        with self.timer.phase("tokenize"):
            ids, sanitized = self.tokenizer.encode_batch_safe(prompts)
        reqs = []
        for p_ids, p in zip(ids, params_list):
            schema = p.guided_decoding.json if p.guided_decoding is not None else None
            with self.timer.phase("fsm_compile"):
                key = self.fsm.compile(schema) if schema is not None else None
            reqs.append(self._make_request(p_ids, p.max_tokens, p.temperature, key))
        with self._cv:
            self.stats["calls"] += 1
            self.stats["prompts_sanitized"] += sanitized
            for r in reqs:
                self.prompt_lens[r.seq.max_new_requested].append(len(r.seq.prompt_ids))
                if r.limit:
                    self.stats[r.limit] += 1
            self._incoming.extend(r for r in reqs if not r.event.is_set())
            self._cv.notify_all()
        return reqs

    def precompile(self, schemas) -> None:
        """Compile + install schemas up front (before serving): no compile inside the timed
        region, and TP followers need not compile a schema the first time it arrives."""
        for schema in schemas:
            key = self.fsm.compile(schema)
            if not self.async_mode:
                with self._device_ctx():
                    self.fsm.install(key)

    def _device_ctx(self):
        return torch.cuda.device(self.device) if self.device.type == "cuda" else contextlib.nullcontext()

    # ---- background scheduler (continuous batching) ----
    def start_async(self):
        """Run the scheduler on a background thread; generate() then only enqueues + waits."""
        if self.async_mode:
            return
        self.async_mode = True
        self._stop = False
        self._thread = threading.Thread(target=self._serve_forever, name="bcg-engine", daemon=True)
        self._thread.start()

    def _serve_forever(self):
        with self._device_ctx():
            while True:
                with self._cv:
                    while not self._stop and not self._incoming and not self._waiting and not any(self.slots):
                        # TP: an idle driver still heartbeats its followers (an empty plan:
                        # their receive must not run into the process-group timeout)
                        if not self._cv.wait(timeout=5.0) and self.tp.size > 1:
                            break
                    if self._stop:
                        break
                try:
                    self._iterate()
                except BaseException as exc:  # fail every pending request loudly
                    self._engine_errors += 1
                    if self._engine_errors <= 3:  # callers may turn it into retries: say what it was
                        import sys
                        import traceback
                        print(f"[engine] scheduler iteration failed ({self._engine_errors}):", file=sys.stderr)
                        traceback.print_exc(file=sys.stderr)
                    self._fail_all(exc)
                    if self.tp.size > 1:  # a TP group cannot re-synchronise after a failed iteration
                        self._stop = True
                        self._fatal = exc
                        break
            if self.tp.size > 1:
                self._release_followers()

    def _release_followers(self):
        """Tell the TP followers to leave their plan loop.  After a failed iteration this is
        best-effort (a follower may be stuck in a collective of that iteration); the error
        rides along so a follower that does receive it raises instead of exiting cleanly."""
        msg = {"stop": True}
        if self._fatal is not None:
            msg["error"] = f"{type(self._fatal).__name__}: {self._fatal}"
        try:
            self._send_plan(msg)
        except Exception:  # noqa: BLE001 -- the control group itself may be gone
            if self._fatal is None:
                raise

    def _fail_all(self, exc):
        self._snap = None
        self._carry = []  # (their slots are failed below)
        with self._cv:
            pending = list(self._incoming) + list(self._waiting)
            self._incoming.clear()
            self._waiting.clear()
        for i, s in enumerate(self.slots):
            if s is not None:
                pending.append(s)
                self.slots[i] = None
        for r in pending:
            r.exc = exc
            r.event.set()

    # ---- TP plan exchange (driver -> followers, CPU group) ----
    def _send_plan(self, plan: dict):
        import torch.distributed as dist
        with self.timer.phase("plan_exchange"):
            dist.broadcast_object_list([plan], src=self.tp.leader, group=self.tp.ctrl)

    def _recv_plan(self) -> dict:
        import torch.distributed as dist
        box = [None]
        with self.timer.phase("plan_wait"):  # follower: includes waiting for the driver's next iteration
            dist.broadcast_object_list(box, src=self.tp.leader, group=self.tp.ctrl)
        return box[0]

    @staticmethod
    def _pack_requests(reqs: List["_Request"]) -> dict:
        lens = [len(r.seq.prompt_ids) for r in reqs]
        ids = np.fromiter((t for r in reqs for t in r.seq.prompt_ids), dtype=np.int32, count=sum(lens))
        return {"ids": ids, "lens": lens, "max_new": [r.seq.max_new for r in reqs],
                "temp": [r.seq.temperature for r in reqs], "fsm": [r.seq.fsm_key for r in reqs]}

    def _unpack_requests(self, spec: dict) -> List["_Request"]:
        reqs, off = [], 0
        ids = spec["ids"].tolist()
        for n, m, t, key in zip(spec["lens"], spec["max_new"], spec["temp"], spec["fsm"]):
            if key is not None:
                with self.timer.phase("fsm_compile"):
                    self.fsm.compile(json.loads(key))
            r = _Request(_Seq(0, ids[off:off + n], m, t, key))
            off += n
            reqs.append(r)
        return reqs

    def serve_follower(self):
        """TP follower loop: apply the driver's plans until it says stop (blocking)."""
        with self._device_ctx():
            while True:
                plan = self._recv_plan()
                if plan.get("stop"):
                    if plan.get("error"):
                        raise RuntimeError(f"TP driver failed: {plan['error']}")
                    return
                self._iterate(plan)

    def start_follower(self):
        """Run `serve_follower` on a background thread (bench / library use)."""
        if self._follower is None:
            self._follower = threading.Thread(target=self._follower_main, name="bcg-tp-follower", daemon=True)
            self._follower.start()

    def _follower_main(self):
        try:
            self.serve_follower()
        except BaseException as exc:  # noqa: BLE001 -- surfaced through `fatal`
            import sys
            import traceback
            print("[engine] TP follower failed:", file=sys.stderr)
            traceback.print_exc(file=sys.stderr)
            self._fatal = exc

    # ---- one scheduler iteration ----
    def _iterate(self, plan: Optional[dict] = None):
        """(TP plan exchange) -> reap -> activate prefills -> admit -> decode burst -> snapshot.

        The host never blocks the device between bursts: completion is read
        from a pinned snapshot taken after the previous burst, and while the
        device is still running that burst the next one is queued FIRST (rows
        that finished in it idle one extra burst, harmlessly -- the sampler
        skips done rows and their blocks are freed only after).  That choice
        depends on timing, so under TP the driver makes it and ships it in the
        plan; followers (``plan`` given) take it from there.
        """
        snap = self._snap
        if plan is None:
            with self._cv:
                new, self._incoming = self._incoming, []
            early = bool(snap is not None and snap["event"] is not None and not snap["event"].query()
                         and self._live_rows())
            if self.tp.size > 1:
                self._send_plan({"new": self._pack_requests(new), "early": early})
        else:
            new = self._unpack_requests(plan["new"])
            early = plan["early"]
        if new:
            for r in new:  # FSM rows are installed here, in admission order (identical on TP ranks)
                if r.seq.fsm_key is not None:
                    r.seq.fsm_base = self.fsm.install(r.seq.fsm_key)
                r.enq_burst = self._bursts
            with self._cv:
                self._waiting.extend(new)
        launched = False
        if early and self._live_rows():
            self._decode_burst()
            launched = True
        self._reap()
        self._admit()
        if not launched and self._live_rows():
            self._decode_burst()
        self._take_snapshot()

    def _take_snapshot(self):
        """Queue a device->pinned-host copy of the completion state of the live rows."""
        rows = self._live_rows()
        if not rows:
            self._snap = None
            return
        n = rows[-1] + 1
        st = self.state
        if self.device.type != "cuda":
            self._snap = {"rows": rows, "n": n, "event": None, "done": st["done"][:n].clone(),
                          "count": st["gen_count"][:n].clone(), "out": st["out_tokens"][:n].clone()}
            return
        if self._snap_buf is None:
            cap = st["done"].shape[0]
            self._snap_buf = {"done": torch.empty(cap, dtype=torch.int32, pin_memory=True),
                              "count": torch.empty(cap, dtype=torch.int32, pin_memory=True),
                              "out": torch.empty(cap, OUT_WIDTH, dtype=torch.int32, pin_memory=True)}
        h = self._snap_buf
        h["done"][:n].copy_(st["done"][:n], non_blocking=True)
        h["count"][:n].copy_(st["gen_count"][:n], non_blocking=True)
        h["out"][:n].copy_(st["out_tokens"][:n], non_blocking=True)
        if self.tp.custom is not None:  # the xGMI all-reduce's timeout word rides along
            if self._ar_err_host is None:
                self._ar_err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
            self.tp.custom.error_async(self._ar_err_host, torch.cuda.current_stream())
        event = torch.cuda.Event()
        event.record()
        self._snap = {"rows": rows, "n": n, "event": event, "done": h["done"], "count": h["count"],
                      "out": h["out"]}

    def _active_rows(self) -> List[int]:
        """Occupied rows (decoding, or pending: prefill in flight)."""
        return [i for i, r in enumerate(self.slots) if r is not None]

    def _live_rows(self) -> List[int]:
        """Rows the decode graphs advance (prefill done)."""
        return [i for i, r in enumerate(self.slots) if r is not None and not r.pending]

    def _admission_deferred(self) -> bool:
        """Admission batching: while the decode batch is well fed, let prompts queue up
        to a full prefill chunk (the prefill GEMMs run at their tuned M instead of
        ragged 2-8k-token tails) -- bounded by `admit_max_wait` bursts of waiting.
        Deterministic under TP: it depends on queue contents and burst counts only."""
        a = self.args
        if a.admit_max_wait <= 0:
            return False
        live = sum(1 for r in self.slots if r is not None and not r.pending)
        if live < a.admit_min_live:
            return False
        if self._bursts - self._waiting[0].enq_burst >= a.admit_max_wait:
            return False
        queued = sum(len(r.seq.prompt_ids) for r in self._waiting)
        queued += sum(len(r.seq.prompt_ids) - r.seq.done_pos for r in self._carry)
        return queued < a.admit_min_tokens_frac * a.prefill_chunk_tokens

    def _hold_tail(self) -> bool:
        """Carry this wave's partial last chunk to the next wave (deterministic under TP: live
        rows and burst counts only): the decode batch is fed and no carried prompt has waited
        past its budget."""
        a = self.args
        if a.prefill_carry_bursts <= 0:
            return False
        live = sum(1 for r in self.slots if r is not None and not r.pending)
        if live < a.admit_min_live:
            return False
        oldest = min((r.enq_burst for r in self._carry), default=self._bursts)
        return self._bursts - oldest < a.admit_max_wait + a.prefill_carry_bursts

    def _admit(self):
        admitted = []
        with self._cv:
            if self._waiting and not self._admission_deferred():
                admitted = self._admit_locked()
        wave, self._carry = self._carry + admitted, []
        if wave and (admitted or not self._hold_tail()):
            self._prefill(wave)
        else:
            self._carry = wave

    def _admit_locked(self) -> List["_Request"]:
        free = [i for i, r in enumerate(self.slots) if r is None]
        cap = self.args.max_batch_seqs
        if self.args.honor_max_num_seqs and self.args.max_num_seqs:
            cap = min(cap, self.args.max_num_seqs)
        budget = max(0, cap - (len(self.slots) - len(free)))
        admitted = []
        while self._waiting and free and len(admitted) < budget:
            req = self._waiting[0]
            a = self.blocks.allocate(req.seq.prompt_ids, req.seq.max_new, self.args.prefix_caching)
            if not a.ok:
                break
            self._waiting.popleft()
            req.seq.blocks, req.seq.cached = list(a.blocks), a.num_cached_tokens
            req.seq.done_pos = a.num_cached_tokens
            req.row = free.pop(0)
            req.pending = True
            self.slots[req.row] = req
            admitted.append(req)
        if not admitted and not any(self.slots) and self._waiting:
            raise RuntimeError("KV cache too small for a single waiting sequence")
        return admitted

    def _prefill(self, wave: List["_Request"]):
        """Prefill the wave's uncached prompt tokens; prompts whose prompt is complete are then
        activated (state rows, prompt blocks committed, token 1 sampled), the others -- their
        tokens in a held partial chunk -- stay pending in the carry."""
        seqs = [r.seq for r in wave]
        table_cpu = self._block_table(seqs, len(seqs))
        with self.timer.phase("prefill"):
            plans = self._plan_prefill(seqs, table_cpu, hold_tail=self._hold_tail())
            logits = self._run_prefill(plans, len(seqs))
        done = [i for i, s in enumerate(seqs) if s.done_pos == len(s.prompt_ids)]
        self._carry = [r for r, s in zip(wave, seqs) if s.done_pos < len(s.prompt_ids)]
        self.stats["prefill_carried"] += len(self._carry)
        if not done:
            return
        if len(done) < len(wave):
            logits = logits.index_select(0, self._h2d(torch.tensor(done, dtype=torch.long)))
        reqs = [wave[i] for i in done]
        seqs = [r.seq for r in reqs]
        table_cpu = table_cpu[done]
        st = self.state
        rows_d = self._h2d(torch.tensor([r.row for r in reqs], dtype=torch.long))
        st["block_tables"].index_copy_(0, rows_d, self._h2d(table_cpu))
        vals = {"seq_lens": [len(s.prompt_ids) for s in seqs], "fsm_base": [s.fsm_base for s in seqs],
                "fsm_state": [0] * len(seqs), "gen_count": [0] * len(seqs),
                "max_new": [s.max_new for s in seqs], "row_keys": [self._next_key() for _ in seqs],
                "done": [0] * len(seqs), "next_tokens": [0] * len(seqs)}
        packed = self._h2d(torch.tensor(list(vals.values()), dtype=torch.int32))  # one upload
        for i, key in enumerate(vals):
            st[key].index_copy_(0, rows_d, packed[i])
        st["temperature"].index_copy_(0, rows_d, self._h2d(torch.tensor([s.temperature for s in seqs],
                                                                         dtype=torch.float32)))
        for s in seqs:  # prompt blocks are now resident: make them reusable
            self.blocks.commit_prompt(s.blocks, s.prompt_ids)
            self.stats["prompt_tokens"] += len(s.prompt_ids)
            self.stats["cached_tokens"] += s.cached
        with self.timer.phase("sample"):
            sub = {k: v.index_select(0, rows_d) for k, v in st.items() if k != "block_tables"}
            self._sample(logits, sub)
            for k, v in sub.items():
                st[k].index_copy_(0, rows_d, v)
        for r in reqs:
            r.pending = False
        self._layout_dirty = True

    def _decode_burst(self):
        """`poll_every` decode steps over the rows [0, bucket)."""
        rows = self._live_rows()
        n = rows[-1] + 1
        if self.cascade is not None and self._layout_dirty:
            self._regroup()
        with self.timer.phase("decode"):
            steps = self.graphs.run_burst(n) if self.graphs is not None else self._eager_burst(n)
        self.stats["decode_steps"] += steps
        self.stats["decode_row_steps"] += steps * len(rows)  # mean live rows = this / decode_steps
        if self.cascade is not None:  # shared tokens read once per group instead of once per row
            self.stats["cascade_shared_row_tokens"] = (self.stats.get("cascade_shared_row_tokens", 0)
                                                       + steps * self.cascade.shared_row_blocks
                                                       * self.args.kv_block_size)
        band = f"rows_le_{1 << max(0, (n - 1).bit_length()) if n <= 512 else (768 if n <= 768 else 1024 if n <= 1024 else 1536)}"
        self.stats[band] = self.stats.get(band, 0) + steps
        self._bursts += 1

    def _regroup(self):
        """Rebuild the shared-prefix tables from the live rows' block lists (engine/cascade.py)."""
        from .cascade import plan_groups
        with self.timer.phase("cascade_plan"):
            rows = [(i, r.seq.blocks) for i, r in enumerate(self.slots) if r is not None and not r.pending]
            self.cascade.upload(plan_groups(rows), self.model.n_q // self.model.n_kv)
        self._layout_dirty = False

    def _eager_burst(self, n: int) -> int:
        view = {k: v[:n] for k, v in self.state.items()}
        for _ in range(self.args.poll_every):
            self.decode_step(view)
        return self.args.poll_every

    def _reap(self):
        """Complete the rows the last snapshot shows finished: detokenise, free KV blocks
        and slots, park and compact (device ops queued behind any burst in flight)."""
        snap, self._snap = self._snap, None
        if snap is None:
            return
        if snap["event"] is not None:
            with self.timer.phase("wait_burst"):
                # sleep-poll instead of hipEventSynchronize, which spins a core for the whole
                # burst (measured: 97 % of the scheduler thread's samples, ~1 core per rank).
                # When the burst is still running the next one is already queued behind it
                # (_iterate's early launch), so the wake-up delay costs no GPU time.
                ev = snap["event"]
                while not ev.query():
                    time.sleep(2e-4)
            if self._ar_err_host is not None and int(self._ar_err_host[0]):
                # a TP peer never arrived at an all-reduce barrier: the activations of
                # this burst are not trustworthy -- fail loudly instead of decoding garbage
                raise RuntimeError("xGMI all-reduce barrier timed out (a tensor-parallel peer stalled or died)")
        n = snap["n"]
        done = snap["done"][:n].tolist()
        finished = [i for i in snap["rows"] if done[i]]
        if not finished:
            return
        counts = snap["count"][:n].tolist()
        with self.timer.phase("detokenize"):
            outs = snap["out"][finished].tolist()
            for i, toks in zip(finished, outs):
                req = self.slots[i]
                toks = toks[:counts[i]]
                if req.seq.fsm_base < 0 and toks and toks[-1] in self.eos_ids:
                    toks = toks[:-1]
                self.stats["generated_tokens"] += counts[i]
                text = self.tokenizer.decode_bytes(toks).decode("utf-8", errors="replace")
                self.blocks.free(req.seq.blocks)
                self.slots[i] = None
                req.finish(text)
        self._park_rows(finished)
        self._layout_dirty = True
        self._compact()

    def _park_rows(self, rows: List[int]):
        """Inactive rows: done, context 1 on the scratch block (harmless in the graph)."""
        if not rows:
            return
        idx = self._h2d(torch.tensor(rows, dtype=torch.long))
        st = self.state
        st["done"].index_fill_(0, idx, 1)
        st["seq_lens"].index_fill_(0, idx, 1)
        st["fsm_base"].index_fill_(0, idx, -1)
        st["block_tables"].index_fill_(0, idx, 0)

    def _compact(self):
        """Move the highest live rows into free low slots when that shrinks the graph bucket.

        Pending rows (prefill in flight) never move: their state is written on activation.
        """
        from .graphs import bucket_for
        occupied = self._active_rows()
        live = self._live_rows()
        if not live:
            return
        if bucket_for(live[-1] + 1) <= bucket_for(len(occupied)):
            return
        free = [i for i in range(len(occupied)) if self.slots[i] is None]
        movers = [i for i in reversed(live) if i >= len(occupied)][:len(free)]
        if not movers:
            return
        src = self._h2d(torch.tensor(movers, dtype=torch.long))
        dst = self._h2d(torch.tensor(free[:len(movers)], dtype=torch.long))
        for key, t in self.state.items():
            t.index_copy_(0, dst, t.index_select(0, src))
        for a, b in zip(movers, free):
            self.slots[b], self.slots[a] = self.slots[a], None
            self.slots[b].row = b
        self._park_rows(movers)

    def _block_table(self, seqs: List[_Seq], rows: int) -> torch.Tensor:
        t = torch.zeros(rows, self.max_blocks_per_seq, dtype=torch.int32)
        for r, s in enumerate(seqs):
            phys = self._phys(s.blocks)
            t[r, :len(phys)] = torch.tensor(phys, dtype=torch.int32)
        return t

    def _next_key(self) -> int:
        self._req_counter += 1
        return (self._req_counter * 0x9E3779B1 + self.seed) & 0x7FFFFFFF

    # ------------------------------------------------------------- prefill
    def _h2d(self, t: torch.Tensor) -> torch.Tensor:
        """Host->device copy that never blocks the host (pinned staging, async on the current stream)."""
        if self.device.type != "cuda":
            return t
        return t.pin_memory().to(self.device, non_blocking=True)

    def _plan_prefill(self, wave: List[_Seq], table_cpu: torch.Tensor, hold_tail: bool = False) -> List[tuple]:
        """Pack the not-yet-prefilled prompt tokens into chunks of exactly `prefill_chunk_tokens`
        (a prompt may straddle chunks; only the last chunk is shorter), so the
        prefill GEMMs run at one M that the shipped tables cover -- M = 16384 is also the one M
        where every projection's 256 x 256 tiles split evenly over 256 CUs.  `hold_tail`: the
        partial last chunk is not run (its prompts keep `done_pos` where it starts).
        Advances each sequence's `done_pos`.  Every chunk's metadata is uploaded before any
        forward is launched."""
        budget = self.args.prefill_chunk_tokens
        plans, chunk, used = [], [], 0
        for r, s in enumerate(wave):
            pos, n = s.done_pos, len(s.prompt_ids)
            while pos < n:
                take = min(n - pos, budget - used)
                chunk.append((r, pos, pos + take))
                used += take
                pos += take
                if used == budget:
                    plans.append(self._plan_chunk(wave, chunk, table_cpu))
                    for rr, _, b in chunk:
                        wave[rr].done_pos = b
                    chunk, used = [], 0
        if chunk and not hold_tail:
            plans.append(self._plan_chunk(wave, chunk, table_cpu))
            for rr, _, b in chunk:
                wave[rr].done_pos = b
            self.stats["prefill_tail_tokens"] += used
        self.stats["prefill_full_chunks"] += len(plans) - (1 if chunk and not hold_tail else 0)
        return plans

    def _plan_chunk(self, wave, chunk, table_cpu):
        bs = self.args.kv_block_size
        toks, pos, slots, q_start, seq_lens, rows, last_idx, last_rows = [], [], [], [0], [], [], [], []
        for r, a, b in chunk:
            s = wave[r]
            toks.extend(s.prompt_ids[a:b])
            p = torch.arange(a, b, dtype=torch.int64)
            pos.append(p)
            phys = table_cpu[r].long()
            slots.append(phys[p // bs] * bs + p % bs)
            q_start.append(q_start[-1] + (b - a))
            seq_lens.append(b)
            rows.append(r)
            if b == len(s.prompt_ids):
                last_idx.append(q_start[-1] - 1)
                last_rows.append(r)
        # query tiles for the HIP prefill kernel (ops.prefill_tile_rows rows), deepest (most keys) first
        tr = self._tile_rows
        tiles = []
        for i, (r, a, b) in enumerate(chunk):
            for t in range(q_start[i], q_start[i + 1], tr):
                tiles.append((b - (q_start[i + 1] - t), i, t, min(t + tr, q_start[i + 1])))
        tiles.sort(key=lambda x: -x[0])
        i32 = torch.int32
        meta = AttnMeta(
            tiles=self._h2d(torch.tensor([x[1:] for x in tiles], dtype=i32)),
            positions=self._h2d(torch.cat(pos).to(i32)),
            slots=self._h2d(torch.cat(slots).to(i32)),
            block_tables=self._h2d(table_cpu[rows]),
            seq_lens=self._h2d(torch.tensor(seq_lens, dtype=i32)),
            q_start=self._h2d(torch.tensor(q_start, dtype=i32)),
            max_q_len=max(b - a for _, a, b in chunk),
            tile_rows=tr,
            decode=False,
            logits_idx=self._h2d(torch.tensor(last_idx if last_idx else [0], dtype=torch.int64)))
        tokens = self._h2d(torch.tensor(toks, dtype=i32))
        dest = self._h2d(torch.tensor(last_rows, dtype=torch.int64)) if last_rows else None
        return tokens, meta, dest, len(last_rows)

    def _run_prefill(self, plans, n_rows: int) -> torch.Tensor:
        """Chunked packed prefill; returns last-token logits ``[n_rows, V]``."""
        logits_out = torch.empty(n_rows, self.model.cfg.vocab_size, dtype=self.args.dtype, device=self.device)
        for tokens, meta, dest, n_last in plans:
            logits = self.model.forward(tokens, meta, self.k_cache, self.v_cache)
            if n_last:
                logits_out.index_copy_(0, dest, logits[:n_last].to(logits_out.dtype))
            self.stats["prefill_chunks"] += 1
        return logits_out

    # -------------------------------------------------------------- decode
    def _sample(self, logits: torch.Tensor, st: Dict[str, torch.Tensor]):
        self.ops.sample_step(logits, self.fsm.table, self.fsm.dist, st["fsm_base"], st["fsm_state"],
                             st["gen_count"], st["max_new"], st["temperature"], st["row_keys"],
                             st["done"], st["seq_lens"], st["out_tokens"], st["next_tokens"],
                             self.seed, self.args.budget_aware_json, self.n_text_tokens,
                             self.eos_ids[0], self.eos_ids[1])

    def decode_meta(self, st: Dict[str, torch.Tensor]) -> AttnMeta:
        bs = self.args.kv_block_size
        pos = (st["seq_lens"] - 1).clamp(min=0)
        rows = torch.arange(pos.shape[0], device=pos.device)
        slots = st["block_tables"][rows, (pos // bs).long()] * bs + pos % bs
        # a finished row idles until the host reaps it (up to ~1.5 bursts): its attention reads one
        # token instead of its whole context (~7 % of decode row-steps; the sampler skips the row)
        attn_lens = None
        if self._skip_done_attn:
            attn_lens = torch.where(st["done"] != 0, torch.ones_like(st["seq_lens"]), st["seq_lens"])
        return AttnMeta(positions=pos, slots=slots.to(torch.int32), block_tables=st["block_tables"],
                        seq_lens=st["seq_lens"], decode=True, workspace=self.decode_ws, cascade=self.cascade,
                        attn_seq_lens=attn_lens)

    def decode_step(self, st: Dict[str, torch.Tensor]):
        """One full decode step (forward + guided sampling), graph-capturable."""
        logits = self.model.forward(st["next_tokens"], self.decode_meta(st), self.k_cache, self.v_cache)
        self._sample(logits, st)

    def shutdown(self):
        self._snap = None
        if self.async_mode:
            with self._cv:
                self._stop = True
                self._cv.notify_all()
            self._thread.join(timeout=120)  # the TP driver's loop sends the followers' stop
            self.async_mode = False
        elif self.tp.size > 1 and self.is_driver and self.model is not None:
            self._release_followers()  # sync-mode driver
        if self._follower is not None:
            self._follower.join(timeout=120)
            self._follower = None
        self.graphs = None
        self.k_cache = self.v_cache = None
        self.model = None


class _Request:
    __slots__ = ("seq", "row", "text", "exc", "event", "pending", "enq_burst", "limit")

    def __init__(self, seq: _Seq, enq_burst: int = 0):
        self.seq, self.row, self.text, self.exc, self.pending = seq, -1, "", None, False
        self.enq_burst = enq_burst
        self.limit = None  # the stats counter of a context-limited request
        self.event = threading.Event()

    def finish(self, text: str):
        self.text = text
        self.event.set()
