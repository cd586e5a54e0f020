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

import hashlib
import json
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


class FakeBackend:
    """Engine backend answering every request with :func:`scripted_text`."""

    name = "fake"

    def __init__(self, seed: int = 0):
        self.seed = seed
        self.calls = 0

    def generate(self, prompts, params_list):
        self.calls += 1
        texts = []
        for prompt, params in zip(prompts, params_list):
            schema = params.guided_decoding.json if params.guided_decoding is not None else None
            texts.append(scripted_text(prompt, schema, self.seed))
        return texts

    def shutdown(self):
        pass
