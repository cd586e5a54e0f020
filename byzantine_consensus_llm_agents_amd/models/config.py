"""Decoder architectures served by the engine (shapes from SURVEY.md §2.3).

One ``ModelConfig`` describes every family the reference can select
(``bcg/config.py:20-25``) plus the plumbing model of BASELINE config 1:

* Qwen3 8B/14B/32B - GQA, per-head QK-RMSNorm, no QKV bias, untied head;
* Qwen2.5-0.5B     - QKV bias, tied embeddings, no QK-norm;
* Mistral-Small-Instruct-2409 (22B) - GQA, no bias, no QK-norm, 32k vocab.

Tiny variants exist for CPU tests.  A model directory with an HF
``config.json`` overrides the preset (``from_hf_config``).
"""

import json
import os
from dataclasses import asdict, dataclass, replace
from typing import Optional


@dataclass(frozen=True)
class ModelConfig:
    name: str
    family: str                 # "qwen3" | "qwen2" | "mistral"
    hidden_size: int
    num_layers: int
    num_heads: int
    num_kv_heads: int
    head_dim: int
    intermediate_size: int
    vocab_size: int             # embedding / lm-head rows
    rope_theta: float = 1_000_000.0
    rms_eps: float = 1e-6
    qk_norm: bool = False
    qkv_bias: bool = False
    tie_embeddings: bool = False
    max_position: int = 32768

    @property
    def q_size(self) -> int:
        return self.num_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_kv_heads * self.head_dim

    def num_params(self) -> int:
        h, i = self.hidden_size, self.intermediate_size
        per_layer = h * (self.q_size + 2 * self.kv_size) + self.q_size * h + 3 * h * i + 2 * h
        if self.qk_norm:
            per_layer += 2 * self.head_dim
        if self.qkv_bias:
            per_layer += self.q_size + 2 * self.kv_size
        emb = self.vocab_size * h * (1 if self.tie_embeddings else 2)
        return per_layer * self.num_layers + emb + h

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return 2 * self.num_layers * self.kv_size * dtype_bytes

    def to_dict(self):
        return asdict(self)


PRESETS = {
    "Qwen/Qwen3-8B": ModelConfig("Qwen/Qwen3-8B", "qwen3", 4096, 36, 32, 8, 128, 12288, 151936,
                                 qk_norm=True, max_position=40960),
    "Qwen/Qwen3-14B": ModelConfig("Qwen/Qwen3-14B", "qwen3", 5120, 40, 40, 8, 128, 17408, 151936,
                                  qk_norm=True, max_position=40960),
    "Qwen/Qwen3-32B": ModelConfig("Qwen/Qwen3-32B", "qwen3", 5120, 64, 64, 8, 128, 25600, 151936,
                                  qk_norm=True, max_position=40960),
    "mistralai/Mistral-Small-Instruct-2409": ModelConfig(
        "mistralai/Mistral-Small-Instruct-2409", "mistral", 6144, 56, 48, 8, 128, 16384, 32768,
        rms_eps=1e-5, max_position=32768),
    "Qwen/Qwen2.5-0.5B-Instruct": ModelConfig("Qwen/Qwen2.5-0.5B-Instruct", "qwen2", 896, 24, 14, 2, 64,
                                              4864, 151936, qkv_bias=True, tie_embeddings=True,
                                              max_position=32768),
    # CPU-test sized variants (same code paths, real tokenizer vocab)
    # (head_dim 64/128 only: the HIP attention kernels are specialised for those)
    "bcg/tiny-qwen3": ModelConfig("bcg/tiny-qwen3", "qwen3", 256, 2, 4, 2, 64, 512, 151936, qk_norm=True),
    "bcg/tiny-qwen2": ModelConfig("bcg/tiny-qwen2", "qwen2", 256, 2, 4, 2, 64, 512, 151936,
                                  qkv_bias=True, tie_embeddings=True),
    "bcg/tiny-mistral": ModelConfig("bcg/tiny-mistral", "mistral", 256, 2, 8, 2, 128, 512, 32768, rms_eps=1e-5),
}

ALIASES = {
    "qwen3-8b": "Qwen/Qwen3-8B",
    "qwen3-14b": "Qwen/Qwen3-14B",
    "qwen3-32b": "Qwen/Qwen3-32B",
    "mistral-22b": "mistralai/Mistral-Small-Instruct-2409",
    "qwen2.5-0.5b": "Qwen/Qwen2.5-0.5B-Instruct",
}


def from_hf_config(path: str, name: Optional[str] = None) -> ModelConfig:
    with open(os.path.join(path, "config.json")) as fh:
        c = json.load(fh)
    arch = (c.get("model_type") or "").lower()
    family = "qwen3" if arch == "qwen3" else ("qwen2" if arch == "qwen2" else "mistral")
    heads = c["num_attention_heads"]
    return ModelConfig(
        name=name or path, family=family, hidden_size=c["hidden_size"],
        num_layers=c["num_hidden_layers"], num_heads=heads,
        num_kv_heads=c.get("num_key_value_heads", heads),
        head_dim=c.get("head_dim") or c["hidden_size"] // heads,
        intermediate_size=c["intermediate_size"], vocab_size=c["vocab_size"],
        rope_theta=float(c.get("rope_theta", 10000.0)), rms_eps=float(c.get("rms_norm_eps", 1e-6)),
        qk_norm=family == "qwen3", qkv_bias=family == "qwen2" or bool(c.get("attention_bias", False)),
        tie_embeddings=bool(c.get("tie_word_embeddings", False)),
        max_position=int(c.get("max_position_embeddings", 32768)))


def get_model_config(name: str, model_dir: Optional[str] = None) -> ModelConfig:
    if model_dir and os.path.exists(os.path.join(model_dir, "config.json")):
        return from_hf_config(model_dir, name)
    key = ALIASES.get(name, name)
    if key in PRESETS:
        return PRESETS[key]
    low = key.lower()
    for preset_name, cfg in PRESETS.items():
        if preset_name.lower() == low:
            return cfg
    raise KeyError(f"unknown model {name!r}; known: {sorted(PRESETS)}")


def with_vocab(cfg: ModelConfig, vocab: int) -> ModelConfig:
    return replace(cfg, vocab_size=vocab)
