"""Native C++ runtime (``csrc/runtime``): token-FSM compiler and KV block manager.

The extension is built in-tree on first import if it is missing or stale, and
a module whose embedded source hash differs from ``csrc/runtime`` is refused.
"""

import importlib

from ..utils.build import build_runtime, runtime_source_hash

build_runtime()
_native = importlib.import_module(__name__ + "._bcg_runtime")
if getattr(_native, "source_hash", None) != runtime_source_hash():
    raise ImportError(f"_bcg_runtime was built from other sources (stamp {getattr(_native, 'source_hash', None)!r}, "
                      f"tree {runtime_source_hash()!r}); rebuild with `python -m "
                      "byzantine_consensus_llm_agents_amd.utils.build --force`")

BlockManager = _native.BlockManager
compile_token_fsm = _native.compile_token_fsm
