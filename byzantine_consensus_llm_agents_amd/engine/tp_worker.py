"""Tensor-parallel follower process (spawned by ``parallel.launcher.spawn_tp_workers``).

Builds the same engine as the driver (its own weight shard, KV cache and
decode graphs on GPU ``LOCAL_RANK``) and replays the driver's scheduling plans
until the driver's engine stops -- the role of a vLLM ``mp`` worker
(``bcg/vllm_agent.py:139-142``).
"""

import json
import os
import sys


def main() -> int:
    spec = json.loads(os.environ["BCG_TP_WORKER_SPEC"])
    from ..bcg.config import ENGINE_CONFIG
    ENGINE_CONFIG.update(spec["engine_config"])
    kw = dict(spec["llm"])
    from .llm import LLM
    llm = LLM(kw.pop("model"), **kw)
    try:
        llm.serve_worker()
    finally:
        llm.backend.shutdown()
        from ..parallel.groups import destroy
        destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
