"""Compatibility module: ``from vllm_agent import VLLMAgent`` keeps working.

The reference's vLLM adapter (``bcg/vllm_agent.py``) is replaced by
:mod:`.engine_agent`; this module only re-exports its names.
"""

from .engine_agent import VERBOSE, EngineAgent, VLLMAgent, extract_json  # noqa: F401
