"""Scripted engine backend: schema-valid JSON without a model.

Used for CPU plumbing runs (BASELINE config 1 without weights) and for the
parity tests, where the *same* function answers both the reference (through a
stub ``vllm`` package, ``tools/gen_golden.py``) and this framework, so that the
two simulators can be diffed on identical engine outputs.

The policy is deterministic in (prompt text, schema, seed) and mildly
"smart" so games actually converge and every termination path is exercised:
honest agents propose the smallest value they can see in their prompt and
vote stop once every proposal shown this round is equal; Byzantine agents
act pseudo-randomly (including abstentions).
"""

import collections
import hashlib
import json
import os
import random
import re
from typing import Any, Dict, Optional

_WORDS = ("consensus value agents agree propose round honest converge keep stable majority "
          "shared initial vote stop continue align group trust evidence signal common").split()

_VALUE_RE = re.compile(r"value: (-?\d+)")
_PROPOSAL_RE = re.compile(r"^  agent_\d+(?: \(you\))?: (-?\d+|ABSTAINED)$", re.M)


def _rng(prompt: str, schema: Optional[Dict], seed: int) -> random.Random:
    h = hashlib.sha256()
    h.update(prompt.encode("utf-8"))
    h.update(json.dumps(schema, sort_keys=True).encode("utf-8"))
    h.update(str(seed).encode())
    return random.Random(int.from_bytes(h.digest()[:8], "little"))


def _sentence(rng: random.Random, n: int) -> str:
    return " ".join(rng.choice(_WORDS) for _ in range(n)).capitalize() + "."


def _enum_of(prop: Dict):
    if "enum" in prop:
        return list(prop["enum"])
    return None


def scripted_object(prompt: str, schema: Optional[Dict], seed: int = 0) -> Any:
    rng = _rng(prompt, schema, seed)
    if not schema or schema.get("type") != "object":
        return {"text": _sentence(rng, 6)}
    props = schema.get("properties", {})
    is_byz = "BYZANTINE" in prompt
    out: Dict[str, Any] = {}
    if "decision" in props:
        options = _enum_of(props["decision"]) or ["stop", "continue"]
        if is_byz:
            out["decision"] = rng.choice(options)
        else:
            shown = _PROPOSAL_RE.findall(prompt)
            nums = [s for s in shown if s != "ABSTAINED"]
            agree = len(nums) > 1 and len(set(nums)) == 1 and len(nums) == len(shown)
            out["decision"] = "stop" if agree else "continue"
        return out
    for name, prop in props.items():
        if name == "value":
            choices = prop.get("anyOf", [prop])
            int_spec = next((c for c in choices if c.get("type") == "integer"), None)
            lo = int_spec.get("minimum", 0) if int_spec else 0
            hi = int_spec.get("maximum", 100) if int_spec else 100
            if is_byz and len(choices) > 1 and rng.random() < 0.2:
                out[name] = "abstain"
            elif is_byz:
                out[name] = rng.randint(lo, hi)
            else:
                seen = [int(v) for v in _VALUE_RE.findall(prompt) if lo <= int(v) <= hi]
                out[name] = min(seen) if seen else rng.randint(lo, hi)
        elif prop.get("type") == "string":
            out[name] = _sentence(rng, rng.randint(3, 12))
    return out


def scripted_text(prompt: str, schema: Optional[Dict], seed: int = 0) -> str:
    return json.dumps(scripted_object(prompt, schema, seed))


# ------------------------------------------------------------ fault injection
_AGENT_RE = re.compile(r"You are (agent_\d+)")
_DECIDE_ROUND_RE = re.compile(r"=== ROUND (\d+) ===")
_VOTE_ROUND_RE = re.compile(r"=== (?:VOTING PHASE|BYZANTINE VOTING) - Round (\d+)/")


class InjectedEngineFault(RuntimeError):
    """Raised by the scripted engine for a call that contains a prompt planned to crash it."""


class FaultInjector:
    """Deterministic engine failures for the retry-ladder parity goldens.

    A plan is a list of rules ``{"agent": "agent_3", "round": 2, "phase":
    "decide"|"vote", "tries": [1, 2], "mode": "invalid_json"|"short"|"exception"}``.
    ``tries`` counts the requests of that (agent, round, phase) in the order
    they are made -- batched attempts, then the sequential attempts (whose
    prompts carry the ``RETRY ATTEMPT k/3`` suffix); ``"all"`` fails every one.  The reference and this
    framework send every agent's requests in the same order, whatever the
    batching, so the same plan fails the same requests on both sides:

    * ``invalid_json`` -- unparsable text (batch and sequential validity fail);
    * ``short``        -- parsable JSON that fails the batched validity rule
      (internal strategy < 3 chars, reasoning < 10) but passes the sequential
      one (non-empty fields); votes: an out-of-enum decision;
    * ``exception``    -- the engine call raises (only meaningful where both
      sides batch identically: homogeneous-schema configurations).
    """

    def __init__(self, plan):
        self.plan = list(plan or [])
        self.tries = collections.Counter()

    @staticmethod
    def identify(prompt: str, schema: Optional[Dict]):
        agent = _AGENT_RE.search(prompt)
        props = (schema or {}).get("properties", {})
        if "decision" in props:
            phase, rnd = "vote", _VOTE_ROUND_RE.search(prompt)
        else:
            phase, rnd = "decide", _DECIDE_ROUND_RE.search(prompt)
        return (agent.group(1) if agent else None, int(rnd.group(1)) if rnd else None, phase)

    def mode_for(self, prompt: str, schema: Optional[Dict]) -> Optional[str]:
        """Count this request and return the planned failure mode (or None)."""
        if not self.plan:
            return None
        key = self.identify(prompt, schema)
        self.tries[key] += 1
        t = self.tries[key]
        for rule in self.plan:
            if (rule["agent"], rule["round"], rule["phase"]) == key and (rule["tries"] == "all" or t in rule["tries"]):
                return rule["mode"]
        return None

    def answer_batch(self, prompts, schemas, seed: int = 0):
        """Texts for one engine call; raises InjectedEngineFault if any prompt plans it."""
        modes = [self.mode_for(p, s) for p, s in zip(prompts, schemas)]
        if "exception" in modes:
            raise InjectedEngineFault("injected engine fault")
        out = []
        for p, s, m in zip(prompts, schemas, modes):
            if m == "invalid_json":
                out.append("I cannot answer in JSON right now {")
            elif m == "short":
                is_vote = "decision" in (s or {}).get("properties", {})
                out.append(json.dumps({"decision": "maybe"} if is_vote else
                                      {"internal_strategy": "ok", "value": 7, "public_reasoning": "short"}))
            else:
                out.append(scripted_text(p, s, seed))
        return out


class FakeBackend:
    """Engine backend answering every request with :func:`scripted_text`."""

    name = "fake"

    def __init__(self, seed: int = 0, faults=None):
        self.seed = seed
        self.calls = 0
        self.delay_s = float(os.environ.get("BCG_FAKE_DELAY_S", "0") or 0)
        if faults is None and os.environ.get("BCG_FAKE_FAULTS"):
            faults = json.loads(os.environ["BCG_FAKE_FAULTS"])
        self.faults = FaultInjector(faults) if faults else None

    def generate(self, prompts, params_list):
        self.calls += 1
        if self.delay_s:  # simulated engine latency per call (load-balance tests)
            import time
            time.sleep(self.delay_s)
        schemas = [p.guided_decoding.json if p.guided_decoding is not None else None for p in params_list]
        if self.faults is not None:
            return self.faults.answer_batch(prompts, schemas, self.seed)
        return [scripted_text(p, s, self.seed) for p, s in zip(prompts, schemas)]

    def shutdown(self):
        pass


class BurnInLLM:
    """Scripted stand-in for :class:`..engine.llm.LLM` used to AGE games before a benchmark.

    ``bench.py`` plays the first rounds of each pool slot's first game with it (CPU
    only, before any timed window), so the timed windows see games of every age --
    as a long-running pool does -- instead of a synchronized fresh start.  Outputs are
    schema-valid (:func:`scripted_object`) with free-text fields padded to the lengths
    the real engine produces (``strategy_chars`` / ``reasoning_chars``; the agents clip
    them to 400 / 600 characters), and every vote is ``continue`` so no game ends
    during burn-in.
    """

    def __init__(self, strategy_chars: int = 400, reasoning_chars: int = 200, seed: int = 0):
        self.strategy_chars, self.reasoning_chars, self.seed = strategy_chars, reasoning_chars, seed
        self.calls = 0

    @staticmethod
    def _text(rng: random.Random, n: int) -> str:
        out = []
        while sum(len(w) + 1 for w in out) < n:
            out.append(rng.choice(_WORDS))
        return " ".join(out)[:n]

    def _answer(self, prompt: str, schema: Optional[Dict]) -> str:
        obj = scripted_object(prompt, schema, self.seed)
        if "decision" in obj:
            obj["decision"] = "continue"
        else:
            rng = _rng(prompt, schema, self.seed + 1)
            if "internal_strategy" in obj:
                obj["internal_strategy"] = self._text(rng, self.strategy_chars)
            if "public_reasoning" in (schema or {}).get("properties", {}):
                obj["public_reasoning"] = self._text(rng, self.reasoning_chars)
        return json.dumps(obj)

    def generate(self, prompts, sampling_params=None, use_tqdm: bool = False):
        from .llm import CompletionOutput, RequestOutput
        if isinstance(prompts, str):
            prompts = [prompts]
        params = sampling_params if isinstance(sampling_params, (list, tuple)) else [sampling_params] * len(prompts)
        self.calls += 1
        outs = []
        for i, (p, sp) in enumerate(zip(prompts, params)):
            schema = sp.guided_decoding.json if sp is not None and sp.guided_decoding is not None else None
            outs.append(RequestOutput(i, p, [CompletionOutput(0, self._answer(p, schema))]))
        return outs


class HostModelBackend:
    """Engine stand-in that does the real engine's HOST work and models its GPU time.

    For measuring whether the host keeps up with several DP ranks per node:
    every call tokenizes its prompts with the model's tokenizer, produces schema-valid outputs
    of the measured mean lengths (:class:`BurnInLLM`; votes drawn by :func:`scripted_object`, so
    games do end), re-tokenizes and detokenizes them (the engine's sampler produces ids, the
    detokenizer text), and waits for a modelled GPU: one FIFO device that processes
    ``tokens_per_s`` (uncached prompt + generated) tokens per second -- the measured rate of the
    real engine -- with ``cached_frac`` of the prompt tokens served by the prefix cache.  The
    real engine batches calls on the device; the model keeps only its throughput, which is what
    the host has to sustain.
    """

    name = "hostmodel"
    async_mode = True  # calls run concurrently (as under continuous batching)

    def __init__(self, model: str, seed: int = 0, tokens_per_s: float = 34000.0, cached_frac: float = 0.375,
                 strategy_chars: int = 310, reasoning_chars: int = 410):
        import threading

        from .tokenizer import load_tokenizer
        self.tok = load_tokenizer(model)
        self.rate, self.cached_frac, self.seed = tokens_per_s, cached_frac, seed
        self.burn = BurnInLLM(strategy_chars, reasoning_chars, seed)
        self.lock = threading.Lock()
        self.free_at = 0.0
        self.stats = {"prompt_tokens": 0, "cached_tokens": 0, "generated_tokens": 0, "calls": 0}
        self.prompt_lens = {}  # prompt token counts per requested max_tokens (as the real engine)
        self.in_flight = 0
        self.closing = threading.Event()
        self.idle = threading.Condition(self.lock)

    def _answer(self, prompt: str, schema: Optional[Dict]) -> str:
        if schema and "decision" in schema.get("properties", {}):
            return json.dumps(scripted_object(prompt, schema, self.seed))
        return self.burn._answer(prompt, schema)

    def generate(self, prompts, params_list):
        import threading
        import time
        if self.closing.is_set():  # after shutdown: park the (daemon) caller in Python, not in native code
            threading.Event().wait()
        t0 = time.perf_counter()
        with self.lock:
            self.in_flight += 1
        try:
            schemas = [p.guided_decoding.json if p.guided_decoding is not None else None for p in params_list]
            p_ids = self.tok.encode_batch(list(prompts))
            out_ids = self.tok.encode_batch([self._answer(p, s) for p, s in zip(prompts, schemas)])
            texts = [self.tok.decode(ids) for ids in out_ids]
        finally:
            with self.lock:
                self.in_flight -= 1
                self.idle.notify_all()
        n_prompt = sum(len(i) for i in p_ids)
        n_cached = int(self.cached_frac * n_prompt)
        n_gen = sum(len(i) for i in out_ids)
        with self.lock:
            start = max(t0, self.free_at)
            self.free_at = start + (n_prompt - n_cached + n_gen) / self.rate
            done = self.free_at
            self.stats["prompt_tokens"] += n_prompt
            self.stats["cached_tokens"] += n_cached
            self.stats["generated_tokens"] += n_gen
            self.stats["calls"] += 1
            for ids, p in zip(p_ids, params_list):
                self.prompt_lens.setdefault(int(p.max_tokens), []).append(len(ids))
        delay = done - time.perf_counter()
        if delay > 0:
            time.sleep(delay)
        return texts

    def shutdown(self):
        # no caller may still be inside the tokenizer's native code when the interpreter
        # finalizes: a daemon thread unwound there aborts the process
        self.closing.set()
        with self.lock:
            self.idle.wait_for(lambda: self.in_flight == 0, timeout=60.0)
