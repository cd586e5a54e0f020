"""L1 LLM adapter: the in-process MI355X engine behind the reference's VLLMAgent API.

Replaces ``bcg/vllm_agent.py`` (``VLLMAgent`` :58-551).  The public surface is
the same -- ``generate``, ``generate_json``, ``batch_generate_json``,
``batch_generate``, ``_format_chat_prompt`` and the class-level ``shutdown`` --
and ``VLLMAgent`` is exported as an alias, so agent code written against the
reference runs unchanged.

The one deliberate behavioural change is the fix of the reference's
batch-size-1 fallback (``vllm_agent.py:417-455``): prompts with *different*
JSON schemas (honest vs Byzantine agents) are still submitted as ONE engine
call, each sequence carrying its own schema FSM on the device.
"""

import gc
import json
import os
from typing import Any, Dict, List, Optional, Tuple

from .chat_templates import format_chat_prompt

VERBOSE = os.environ.get("VERBOSE", "0") == "1"

_DEFAULT_MODEL_CONFIG = {
    "max_model_len": 4096,
    "gpu_memory_utilization": 0.85,
    "tensor_parallel_size": 1,
    "max_num_seqs": 64,
}


def extract_json(text: str) -> Optional[Dict[str, Any]]:
    """First balanced ``{...}`` span of ``text`` that parses as JSON."""
    start = text.find("{")
    if start < 0:
        return None
    depth = 0
    for i in range(start, len(text)):
        ch = text[i]
        if ch == "{":
            depth += 1
        elif ch == "}":
            depth -= 1
            if depth == 0:
                try:
                    return json.loads(text[start:i + 1])
                except (json.JSONDecodeError, ValueError):
                    pass
    return None


def _clean(text: str) -> str:
    text = text.strip()
    while text.startswith("\n"):
        text = text[1:].strip()
    return text


def parse_single(text: str) -> Dict[str, Any]:
    """Parsing used by ``generate_json`` (reference :332-369)."""
    text = _clean(text)
    try:
        return json.loads(text)
    except json.JSONDecodeError:
        pass
    obj = extract_json(text)
    if obj is not None:
        return obj
    return {"error": "json_parse_failed",
            "message": "Could not extract valid JSON from model output", "raw": text[:200]}


def parse_batched(text: str) -> Dict[str, Any]:
    """Parsing used by the batched path (reference :433-441)."""
    text = text.strip()
    try:
        return json.loads(text)
    except json.JSONDecodeError:
        obj = extract_json(text)
        return obj if obj else {"error": "json_parse_failed", "raw": text[:100]}


class EngineAgent:
    """Agent base class sharing one in-process inference engine."""

    _shared_llm = None
    _shared_model_name: Optional[str] = None
    _shared_model_config: Optional[Dict[str, Any]] = None

    def __init__(self, agent_id: str, model_name: str = "Qwen/Qwen3-8B",
                 model_config: Optional[Dict[str, Any]] = None):
        self.agent_id = agent_id
        self.model_name = model_name
        self.model_config = model_config or dict(_DEFAULT_MODEL_CONFIG)
        cls = EngineAgent
        if (cls._shared_llm is None or cls._shared_model_name != model_name
                or cls._shared_model_config != self.model_config):
            self._load_model()
        self.llm = cls._shared_llm

    # ------------------------------------------------------------- engine
    def _load_model(self):
        from ..engine.llm import LLM  # local import: keeps the bcg layer importable alone
        cfg = self.model_config
        if VERBOSE:
            print(f"Loading model {self.model_name}...", flush=True)
        for key, value in cfg.get("env_vars", {}).items():
            os.environ[key] = value
        if EngineAgent._shared_llm is not None:
            EngineAgent._shared_llm.shutdown()
        EngineAgent._shared_llm = LLM(
            model=self.model_name,
            max_model_len=cfg.get("max_model_len", 8192),
            gpu_memory_utilization=cfg.get("gpu_memory_utilization", 0.85),
            tensor_parallel_size=cfg.get("tensor_parallel_size", 1),
            max_num_seqs=cfg.get("max_num_seqs"),
            quantization=cfg.get("quantization"),
        )
        EngineAgent._shared_model_name = self.model_name
        EngineAgent._shared_model_config = dict(cfg)

    @staticmethod
    def _params(temperature, max_tokens, top_p=1.0, schema=None):
        from ..engine.llm import GuidedDecodingParams, SamplingParams
        guided = GuidedDecodingParams(json=schema) if schema is not None else None
        return SamplingParams(temperature=temperature, top_p=top_p, max_tokens=max_tokens,
                              guided_decoding=guided)

    def _format_chat_prompt(self, system_prompt: str, user_prompt: str) -> str:
        return format_chat_prompt(self.model_name, self.model_config, system_prompt, user_prompt)

    # ----------------------------------------------------------- text APIs
    def generate(self, prompt: str, temperature: float = 0.0, max_tokens: int = 256,
                 top_p: float = 1.0, system_prompt: Optional[str] = None, **kwargs) -> str:
        full = self._format_chat_prompt(system_prompt, prompt) if system_prompt else prompt
        out = self.llm.generate([full], self._params(temperature, max_tokens, top_p))
        return out[0].outputs[0].text.strip()

    def batch_generate(self, prompts: List[str], temperature: float = 0.0, max_tokens: int = 256,
                       top_p: float = 1.0, **kwargs) -> List[str]:
        outs = self.llm.generate(list(prompts), self._params(temperature, max_tokens, top_p))
        return [o.outputs[0].text.strip() for o in outs]

    # ----------------------------------------------------------- JSON APIs
    def generate_json(self, prompt: str, schema: Dict[str, Any], temperature: float = 0.0,
                      max_tokens: int = 512, system_prompt: Optional[str] = None) -> Dict[str, Any]:
        try:
            full = self._format_chat_prompt(system_prompt, prompt) if system_prompt else prompt
            out = self.llm.generate([full], self._params(temperature, max_tokens, schema=schema))
            return parse_single(out[0].outputs[0].text)
        except Exception as exc:  # engine faults become per-prompt errors (reference :376-379)
            if VERBOSE:
                print(f"⚠️ JSON generation failed: {exc}")
            return {"error": str(exc), "message": "JSON generation failed"}

    def batch_generate_json(self, prompts: List[Tuple[str, str, Dict[str, Any]]],
                            temperature: float = 0.8, max_tokens: int = 512) -> List[Dict[str, Any]]:
        """One engine call for all prompts, heterogeneous schemas included."""
        if not prompts:
            return []
        texts = [self._format_chat_prompt(s, u) for s, u, _ in prompts]
        params = [self._params(temperature, max_tokens, schema=sch) for _, _, sch in prompts]
        homogeneous = all(sch == prompts[0][2] for _, _, sch in prompts)
        try:
            outs = self.llm.generate(texts, params)
        except Exception as exc:
            if VERBOSE:
                print(f"⚠️ Batched JSON generation failed: {exc}")
            if homogeneous:
                return [{"error": str(exc)} for _ in prompts]
            return [{"error": str(exc), "message": "JSON generation failed"} for _ in prompts]
        parse = parse_batched if homogeneous else parse_single
        return [parse(o.outputs[0].text) for o in outs]

    _extract_json = staticmethod(extract_json)

    # ------------------------------------------------------------ teardown
    @classmethod
    def shutdown(cls):
        if EngineAgent._shared_llm is not None:
            try:
                EngineAgent._shared_llm.shutdown()
            except Exception:
                pass
        EngineAgent._shared_llm = None
        EngineAgent._shared_model_name = None
        EngineAgent._shared_model_config = None
        gc.collect()
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.synchronize()
                torch.cuda.empty_cache()
                torch.cuda.reset_peak_memory_stats()
        except Exception:
            pass
        try:
            import torch.distributed as dist
            if dist.is_initialized():
                dist.destroy_process_group()
        except Exception:
            pass
        gc.collect()


# API-compatible alias for code written against the reference.
VLLMAgent = EngineAgent
