"""In-process inference engine (replaces the reference's vLLM dependency)."""

from .llm import LLM, CompletionOutput, GuidedDecodingParams, RequestOutput, SamplingParams  # noqa: F401
