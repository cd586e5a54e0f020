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
"""

import math
import os
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch

from ..bcg.config import ENGINE_CONFIG
from ..models.config import ModelConfig, get_model_config
from ..models.transformer import AttnMeta, DecoderModel, TPGroup
from ..ops import get_ops
from ..utils.trace import PhaseTimer
from .guided.compiler import FSMRegistry
from .tokenizer import load_tokenizer


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
    max_whitespace: int = 4
    prefix_caching: bool = True
    use_hip_graphs: bool = True
    kv_cache_gb: Optional[float] = None
    honor_max_num_seqs: bool = False
    dtype: torch.dtype = torch.bfloat16
    device: Optional[str] = None
    poll_every: int = 8

    @classmethod
    def from_configs(cls, model: str, backend: str, weights: Optional[str] = None,
                     seed: Optional[int] = None, **kw) -> "EngineArgs":
        ec = ENGINE_CONFIG
        weights = weights or ec.get("weights") or "auto"
        model_dir = weights if weights not in ("auto", "random") else None
        cfg = get_model_config(model, model_dir)
        args = cls(model=model, model_cfg=cfg, backend=backend,
                   weights="random" if weights == "auto" else weights, seed=seed,
                   kv_block_size=ec.get("kv_block_size", 16),
                   max_batch_seqs=ec.get("max_batch_seqs", 512),
                   prefill_chunk_tokens=ec.get("prefill_chunk_tokens", 16384),
                   budget_aware_json=ec.get("budget_aware_json", False),
                   max_whitespace=ec.get("max_whitespace", 4),
                   prefix_caching=ec.get("prefix_caching", True),
                   use_hip_graphs=ec.get("use_hip_graphs", True),
                   kv_cache_gb=ec.get("kv_cache_gb"),
                   honor_max_num_seqs=ec.get("honor_max_num_seqs", False))
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
    fsm_base: int
    blocks: List[int] = field(default_factory=list)
    cached: int = 0
    error: Optional[str] = None


class InferenceEngine:
    def __init__(self, args: EngineArgs):
        self.args = args
        self.timer = PhaseTimer()
        self.stats = {"prompt_tokens": 0, "cached_tokens": 0, "generated_tokens": 0,
                      "decode_steps": 0, "prefill_chunks": 0, "calls": 0}
        cfg = args.model_cfg
        self.backend = args.backend
        if args.device:
            self.device = torch.device(args.device)
        elif self.backend == "hip":
            if not torch.cuda.is_available():
                raise RuntimeError("hip backend requested but no GPU is visible")
            self.device = torch.device("cuda", torch.cuda.current_device())
        else:
            self.device = torch.device("cpu")
        self.tp = self._init_tp(args.tensor_parallel_size)
        self.ops = get_ops(self.backend)

        model_dir = args.weights if args.weights not in ("random", "auto") else None
        self.tokenizer = load_tokenizer(args.model, model_dir)
        if self.tokenizer.vocab_size > cfg.vocab_size:
            raise ValueError("tokenizer larger than the model vocabulary")
        self.model = DecoderModel(cfg, self.ops, self.device, args.dtype, self.tp)
        with self.timer.phase("load_weights"):
            if model_dir:
                from ..models.loader import load_safetensors_dir
                self.model.load_hf_state_dict(load_safetensors_dir(model_dir))
            else:
                self.model.init_random(seed=args.seed or 0)
        self.seed = (args.seed if args.seed is not None else int.from_bytes(os.urandom(4), "little")) & 0x7FFFFFFF
        self._req_counter = 0

        self.fsm = FSMRegistry(self.tokenizer.all_token_bytes(), cfg.vocab_size, self.device,
                               max_ws=args.max_whitespace)
        self.eos_ids = (self.tokenizer.eos_token_ids + [self.tokenizer.eos_token_ids[0]])[:2]
        self.n_text_tokens = min(self.tokenizer.vocab_size, cfg.vocab_size)
        self._alloc_kv_cache()
        if self.backend == "hip":
            self._load_tuned_gemms()
        self.graphs = None
        if self.backend == "hip" and args.use_hip_graphs:
            from .graphs import DecodeGraphs
            self.graphs = DecodeGraphs(self)

    # ------------------------------------------------------------- setup
    def _init_tp(self, tp_size: int) -> TPGroup:
        if tp_size <= 1:
            return TPGroup()
        from ..parallel.groups import tensor_parallel_group
        return tensor_parallel_group(tp_size)

    def _alloc_kv_cache(self):
        a, m = self.args, self.model
        bs = a.kv_block_size
        per_block = 2 * m.cfg.num_layers * m.n_kv * bs * m.hd * torch.tensor([], dtype=a.dtype).element_size()
        want_tokens = a.max_batch_seqs * a.max_model_len
        if a.kv_cache_gb:
            budget = int(a.kv_cache_gb * 2 ** 30)
        elif self.device.type == "cuda":
            free, total = torch.cuda.mem_get_info(self.device)
            reserve = 6 * 2 ** 30 + 2 * a.prefill_chunk_tokens * (m.cfg.hidden_size + 2 * m.inter) * 2
            budget = int(min(free - reserve, total * a.gpu_memory_utilization - torch.cuda.memory_allocated(self.device)))
        else:
            budget = 256 * 2 ** 20
        num_blocks = max(16, min(budget // per_block, want_tokens // bs + 1))
        self.k_cache = torch.zeros((m.cfg.num_layers, num_blocks, m.n_kv, bs, m.hd), dtype=a.dtype,
                                   device=self.device)
        # V is stored transposed per block-head (see ops/reference.py)
        self.v_cache = torch.zeros((m.cfg.num_layers, num_blocks, m.n_kv, m.hd, bs), dtype=a.dtype,
                                   device=self.device)
        from ..runtime import BlockManager
        # block 0 is scratch (padding rows of graph buckets write there); never handed out
        self.blocks = BlockManager(num_blocks - 1, bs)
        self.num_blocks = num_blocks
        self.max_blocks_per_seq = (a.max_model_len + bs - 1) // bs
        self.kv_bytes = 2 * self.k_cache.numel() * self.k_cache.element_size()

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

    def _phys(self, blocks: List[int]) -> List[int]:
        return [b + 1 for b in blocks]  # manager ids are shifted past scratch block 0

    # ------------------------------------------------------------ serving
    def generate(self, prompts: List[str], params_list) -> List[str]:
        # the coalescer may run this on any simulation thread; the current HIP
        # device (and with it torch.cuda.current_stream used by the ctypes
        # launches) is thread-local, so pin it for the whole call
        if self.device.type == "cuda":
            with torch.cuda.device(self.device):
                return self._generate(prompts, params_list)
        return self._generate(prompts, params_list)

    def _generate(self, prompts: List[str], params_list) -> List[str]:
        self.stats["calls"] += 1
        with self.timer.phase("tokenize"):
            ids = self.tokenizer.encode_batch(prompts)
        seqs: List[_Seq] = []
        for i, (p_ids, p) in enumerate(zip(ids, params_list)):
            schema = p.guided_decoding.json if p.guided_decoding is not None else None
            with self.timer.phase("fsm_compile"):
                base = self.fsm.get(schema) if schema is not None else -1
            s = _Seq(i, p_ids, max(1, int(p.max_tokens)), float(p.temperature), base)
            if len(p_ids) == 0 or len(p_ids) + s.max_new > self.args.max_model_len:
                s.error = "prompt too long" if p_ids else "empty prompt"
            seqs.append(s)
        texts = [""] * len(seqs)
        todo = [s for s in seqs if s.error is None]
        wave_cap = self.args.max_batch_seqs
        if self.args.honor_max_num_seqs and self.args.max_num_seqs:
            wave_cap = min(wave_cap, self.args.max_num_seqs)
        while todo:
            wave, todo = self._admit(todo, wave_cap)
            if not wave:
                raise RuntimeError("KV cache too small for a single sequence")
            for s, text in zip(wave, self._run_wave(wave)):
                texts[s.idx] = text
        return texts

    def _admit(self, todo: List[_Seq], cap: int):
        admitted, rest = [], []
        for s in todo:
            if len(admitted) >= cap:
                rest.append(s)
                continue
            a = self.blocks.allocate(s.prompt_ids, s.max_new, self.args.prefix_caching)
            if not a.ok:
                rest.append(s)
                continue
            s.blocks, s.cached = list(a.blocks), a.num_cached_tokens
            admitted.append(s)
        return admitted, rest

    def _block_table(self, wave: List[_Seq], rows: int) -> torch.Tensor:
        t = torch.zeros(rows, self.max_blocks_per_seq, dtype=torch.int32)
        for r, s in enumerate(wave):
            phys = self._phys(s.blocks)
            t[r, :len(phys)] = torch.tensor(phys, dtype=torch.int32)
        return t

    def _run_wave(self, wave: List[_Seq]) -> List[str]:
        B = len(wave)
        dev = self.device
        bs = self.args.kv_block_size
        max_new = max(s.max_new for s in wave)
        table_cpu = self._block_table(wave, B)
        st = {
            "block_tables": table_cpu.to(dev),
            "seq_lens": torch.tensor([len(s.prompt_ids) for s in wave], dtype=torch.int32, device=dev),
            "fsm_base": torch.tensor([s.fsm_base for s in wave], dtype=torch.int32, device=dev),
            "fsm_state": torch.zeros(B, dtype=torch.int32, device=dev),
            "gen_count": torch.zeros(B, dtype=torch.int32, device=dev),
            "max_new": torch.tensor([s.max_new for s in wave], dtype=torch.int32, device=dev),
            "temperature": torch.tensor([s.temperature for s in wave], dtype=torch.float32, device=dev),
            "row_keys": torch.tensor([self._next_key() for _ in wave], dtype=torch.int32, device=dev),
            "done": torch.zeros(B, dtype=torch.int32, device=dev),
            "next_tokens": torch.zeros(B, dtype=torch.int32, device=dev),
            "out_tokens": torch.zeros(B, max_new, dtype=torch.int32, device=dev),
        }
        with self.timer.phase("prefill"):
            logits = self._prefill(wave, table_cpu, st["block_tables"])
        for s in wave:  # prompt blocks are now resident: make them reusable
            self.blocks.commit_prompt(s.blocks, s.prompt_ids)
        with self.timer.phase("sample"):
            self._sample(logits, st)
        with self.timer.phase("decode"):
            self._decode(st, B, max_new)
        with self.timer.phase("detokenize"):
            counts = st["gen_count"].cpu().tolist()
            outs = st["out_tokens"].cpu().tolist()
            texts = []
            for r, s in enumerate(wave):
                toks = outs[r][:counts[r]]
                if s.fsm_base < 0 and toks and toks[-1] in self.eos_ids:
                    toks = toks[:-1]
                self.stats["generated_tokens"] += counts[r]
                texts.append(self.tokenizer.decode_bytes(toks).decode("utf-8", errors="replace"))
        for s in wave:
            self.blocks.free(s.blocks)
            self.stats["prompt_tokens"] += len(s.prompt_ids)
            self.stats["cached_tokens"] += s.cached
        return texts

    def _next_key(self) -> int:
        self._req_counter += 1
        x = (self._req_counter * 0x9E3779B1 + self.seed) & 0x7FFFFFFF
        return x

    # ------------------------------------------------------------- prefill
    def _prefill(self, wave: List[_Seq], table_cpu: torch.Tensor, table_dev: torch.Tensor) -> torch.Tensor:
        """Chunked packed prefill; returns last-token logits ``[B, V]``."""
        dev, bs = self.device, self.args.kv_block_size
        V = self.model.cfg.vocab_size
        logits_out = torch.empty(len(wave), V, dtype=self.args.dtype, device=dev)
        budget = self.args.prefill_chunk_tokens
        # (row, start, end) segments of uncached prompt tokens
        segments = []
        for r, s in enumerate(wave):
            pos, n = s.cached, len(s.prompt_ids)
            while pos < n:
                end = min(n, pos + budget)
                segments.append((r, pos, end))
                pos = end
        chunk, used = [], 0
        for seg in segments + [None]:
            if seg is not None and used + (seg[2] - seg[1]) <= budget:
                chunk.append(seg)
                used += seg[2] - seg[1]
                continue
            if chunk:
                self._prefill_chunk(wave, chunk, table_cpu, logits_out)
            chunk, used = ([seg], seg[2] - seg[1]) if seg is not None else ([], 0)
        return logits_out

    def _prefill_chunk(self, wave, chunk, table_cpu, logits_out):
        dev, bs = self.device, self.args.kv_block_size
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
        # 64-query tiles for the HIP prefill kernel, deepest (most keys) first
        tiles = []
        for i, (r, a, b) in enumerate(chunk):
            for t in range(q_start[i], q_start[i + 1], 64):
                tiles.append((b - (q_start[i + 1] - t), i, t, min(t + 64, q_start[i + 1])))
        tiles.sort(key=lambda x: -x[0])
        meta = AttnMeta(
            tiles=torch.tensor([x[1:] for x in tiles], dtype=torch.int32, device=dev),
            positions=torch.cat(pos).to(torch.int32).to(dev),
            slots=torch.cat(slots).to(torch.int32).to(dev),
            block_tables=table_cpu[rows].to(dev),
            seq_lens=torch.tensor(seq_lens, dtype=torch.int32, device=dev),
            q_start=torch.tensor(q_start, dtype=torch.int32, device=dev),
            max_q_len=max(b - a for _, a, b in chunk),
            decode=False,
            logits_idx=torch.tensor(last_idx if last_idx else [0], dtype=torch.int64, device=dev))
        tokens = torch.tensor(toks, dtype=torch.int32, device=dev)
        logits = self.model.forward(tokens, meta, self.k_cache, self.v_cache)
        if last_rows:
            logits_out[torch.tensor(last_rows, device=dev)] = logits[:len(last_rows)].to(logits_out.dtype)
        self.stats["prefill_chunks"] += 1

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
        return AttnMeta(positions=pos, slots=slots.to(torch.int32), block_tables=st["block_tables"],
                        seq_lens=st["seq_lens"], decode=True)

    def decode_step(self, st: Dict[str, torch.Tensor]):
        """One full decode step (forward + guided sampling), graph-capturable."""
        logits = self.model.forward(st["next_tokens"], self.decode_meta(st), self.k_cache, self.v_cache)
        self._sample(logits, st)

    def _decode(self, st: Dict[str, torch.Tensor], B: int, max_new: int):
        steps = 0
        if self.graphs is not None:
            steps = self.graphs.run(st, B, max_new)
        else:
            poll = self.args.poll_every
            for i in range(1, max_new):
                if i % poll == 1 and bool(st["done"].all()):
                    break
                self.decode_step(st)
                steps += 1
        self.stats["decode_steps"] += steps

    def shutdown(self):
        self.graphs = None
        self.k_cache = self.v_cache = None
        self.model = None
