"""HF checkpoint IO: safetensors (single file or sharded with an index), config.json.

The reference hands the model name to vLLM, which downloads and loads the HF
checkpoint (``bcg/vllm_agent.py:126-144``).  There is no network here, so the
engine loads a local directory (``ENGINE_CONFIG["weights"]`` / ``--weights``)
and otherwise random-initialises the architecture.  Only safetensors are
read (no pickle): ``safetensors.safe_open`` memory-maps each shard and
tensors are materialised one at a time, so a TP rank slices its shard
without holding the full checkpoint in host memory twice.
"""

import json
import os
from typing import Dict, Iterable, Optional

import torch

from .config import ModelConfig


def _shard_files(model_dir: str) -> Iterable[str]:
    index = os.path.join(model_dir, "model.safetensors.index.json")
    if os.path.exists(index):
        with open(index) as fh:
            files = sorted(set(json.load(fh)["weight_map"].values()))
        return [os.path.join(model_dir, f) for f in files]
    files = sorted(f for f in os.listdir(model_dir) if f.endswith(".safetensors"))
    if not files:
        raise FileNotFoundError(f"no *.safetensors under {model_dir}")
    return [os.path.join(model_dir, f) for f in files]


class LazyStateDict(dict):
    """name -> tensor, loaded from the memory-mapped shards on first access."""

    def __init__(self, model_dir: str):
        super().__init__()
        from safetensors import safe_open
        self._where = {}
        self._handles = {}
        for path in _shard_files(model_dir):
            h = safe_open(path, framework="pt", device="cpu")
            self._handles[path] = h
            for k in h.keys():
                self._where[k] = path

    def __contains__(self, key) -> bool:
        return key in self._where

    def __getitem__(self, key) -> torch.Tensor:
        return self._handles[self._where[key]].get_tensor(key)

    def keys(self):
        return self._where.keys()

    def __iter__(self):
        return iter(self._where)

    def __len__(self) -> int:
        return len(self._where)


def load_safetensors_dir(model_dir: str) -> LazyStateDict:
    return LazyStateDict(model_dir)


def hf_config_dict(cfg: ModelConfig) -> Dict:
    model_type = {"qwen3": "qwen3", "qwen2": "qwen2", "mistral": "mistral"}[cfg.family]
    return {
        "model_type": model_type, "hidden_size": cfg.hidden_size, "num_hidden_layers": cfg.num_layers,
        "num_attention_heads": cfg.num_heads, "num_key_value_heads": cfg.num_kv_heads,
        "head_dim": cfg.head_dim, "intermediate_size": cfg.intermediate_size, "vocab_size": cfg.vocab_size,
        "rope_theta": cfg.rope_theta, "rms_norm_eps": cfg.rms_eps, "tie_word_embeddings": cfg.tie_embeddings,
        "max_position_embeddings": cfg.max_position, "attention_bias": cfg.qkv_bias,
        "torch_dtype": "bfloat16",
    }


def save_hf_checkpoint(state_dict: Dict[str, torch.Tensor], cfg: ModelConfig, model_dir: str,
                       max_shard_bytes: Optional[int] = None):
    """Write config.json + safetensors (sharded with an index when max_shard_bytes is set)."""
    from safetensors.torch import save_file
    os.makedirs(model_dir, exist_ok=True)
    with open(os.path.join(model_dir, "config.json"), "w") as fh:
        json.dump(hf_config_dict(cfg), fh, indent=1)
    sd = {k: v.detach().contiguous().cpu() for k, v in state_dict.items()}
    if not max_shard_bytes:
        save_file(sd, os.path.join(model_dir, "model.safetensors"))
        return
    shards, cur, size = [], {}, 0
    for k, v in sd.items():
        nbytes = v.numel() * v.element_size()
        if cur and size + nbytes > max_shard_bytes:
            shards.append(cur)
            cur, size = {}, 0
        cur[k] = v
        size += nbytes
    if cur:
        shards.append(cur)
    weight_map = {}
    for i, shard in enumerate(shards):
        name = f"model-{i + 1:05d}-of-{len(shards):05d}.safetensors"
        save_file(shard, os.path.join(model_dir, name))
        weight_map.update({k: name for k in shard})
    with open(os.path.join(model_dir, "model.safetensors.index.json"), "w") as fh:
        json.dump({"metadata": {}, "weight_map": weight_map}, fh, indent=1)
