import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.device_count() > 0
    except Exception:
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU visible")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture
def fresh_engine_state():
    """Reset config dicts and the shared engine between tests."""
    from byzantine_consensus_llm_agents_amd.bcg import config as cfg
    from byzantine_consensus_llm_agents_amd.bcg.engine_agent import EngineAgent
    saved = {name: dict(getattr(cfg, name)) for name in
             ("BCG_CONFIG", "VLLM_CONFIG", "AGENT_CONFIG", "METRICS_CONFIG", "ENGINE_CONFIG",
              "NETWORK_CONFIG", "LLM_CONFIG")}
    EngineAgent.shutdown()
    yield cfg
    EngineAgent.shutdown()
    for name, value in saved.items():
        d = getattr(cfg, name)
        d.clear()
        d.update(value)
