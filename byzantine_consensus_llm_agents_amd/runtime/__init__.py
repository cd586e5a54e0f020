"""Native C++ runtime (``csrc/runtime``): token-FSM compiler and KV block manager.

The extension is built in-tree on first import if it is missing or stale.
"""

import importlib

from ..utils.build import build_runtime

build_runtime()
_native = importlib.import_module(__name__ + "._bcg_runtime")

BlockManager = _native.BlockManager
compile_token_fsm = _native.compile_token_fsm
