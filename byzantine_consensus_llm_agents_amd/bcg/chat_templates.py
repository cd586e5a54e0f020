"""Raw chat templates used by the agents (reference ``bcg/vllm_agent.py:199-292``).

The reference formats prompts with hand-written templates (not HF
``apply_chat_template``); the bytes matter for parity, so they are reproduced
here as a table keyed by model family.  Qwen3 appends `` /no_think`` to the
user turn unless the model is an Instruct-2507 variant or
``disable_qwen3_thinking`` is False.
"""

from typing import Dict, Optional

CHATML = "<|im_start|>system\n{system}<|im_end|>\n<|im_start|>user\n{user}<|im_end|>\n<|im_start|>assistant\n"
CHATML_NO_THINK = "<|im_start|>system\n{system}<|im_end|>\n<|im_start|>user\n{user} /no_think<|im_end|>\n<|im_start|>assistant\n"
LLAMA3 = ("<|begin_of_text|><|start_header_id|>system<|end_header_id|>\n\n{system}<|eot_id|>"
          "<|start_header_id|>user<|end_header_id|>\n\n{user}<|eot_id|>"
          "<|start_header_id|>assistant<|end_header_id|>\n\n")
LLAMA2_INST = "<s>[INST] <<SYS>>\n{system}\n<</SYS>>\n\n{user} [/INST]"


def template_family(model_name: str, model_config: Optional[Dict] = None) -> str:
    """Name of the template the reference would pick for ``model_name``."""
    name = model_name.lower()
    cfg = model_config or {}
    if "qwen3" in name or "qwen-3" in name:
        if "instruct-2507" in name or "instruct_2507" in name:
            return "qwen3_2507"
        return "qwen3_no_think" if cfg.get("disable_qwen3_thinking", True) else "qwen3_think"
    if "qwen" in name:
        return "qwen2"
    if "llama-3" in name or "llama3" in name:
        return "llama3"
    if "llama" in name or "mistral" in name:
        return "llama2_inst"
    return "chatml"


_TEMPLATES = {
    "qwen3_2507": CHATML,
    "qwen3_no_think": CHATML_NO_THINK,
    "qwen3_think": CHATML,
    "qwen2": CHATML,
    "llama3": LLAMA3,
    "llama2_inst": LLAMA2_INST,
    "chatml": CHATML,
}


def format_chat_prompt(model_name: str, model_config: Optional[Dict],
                       system_prompt: str, user_prompt: str) -> str:
    # plain concatenation (not str.format) so braces inside prompts are safe
    tpl = _TEMPLATES[template_family(model_name, model_config)]
    head, rest = tpl.split("{system}", 1)
    mid, tail = rest.split("{user}", 1)
    return head + system_prompt + mid + user_prompt + tail


def system_prefix(model_name: str, model_config: Optional[Dict], system_prompt: str) -> str:
    """The part of the formatted prompt that depends only on the system prompt.

    Used by the engine's prefix cache: everything up to and including the
    user-turn header is identical across rounds for a given agent.
    """
    tpl = _TEMPLATES[template_family(model_name, model_config)]
    head, rest = tpl.split("{system}", 1)
    mid = rest.split("{user}", 1)[0]
    return head + system_prompt + mid
