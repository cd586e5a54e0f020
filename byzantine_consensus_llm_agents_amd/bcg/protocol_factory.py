"""Protocol factory (reference ``bcg/protocol_factory.py:11-44``).

A registry instead of an if-chain so new protocols can be plugged in with
:func:`register_protocol`; ``"a2a_sim"`` is registered by default and an
unknown name raises ``ValueError`` with the same message shape.
"""

from typing import Any, Callable, Dict, List, Optional

from .a2a_sim import A2ASimProtocol
from .communication_protocol import CommunicationProtocol

_REGISTRY: Dict[str, Callable[..., CommunicationProtocol]] = {}


def register_protocol(name: str, ctor: Callable[..., CommunicationProtocol]) -> None:
    _REGISTRY[name] = ctor


register_protocol("a2a_sim", lambda num_agents, topology, config:
                  A2ASimProtocol(num_agents=num_agents, topology=topology))


def create_protocol(protocol_type: str, num_agents: int, topology: Dict[int, List[int]],
                    config: Optional[Dict[str, Any]] = None) -> CommunicationProtocol:
    ctor = _REGISTRY.get(protocol_type)
    if ctor is None:
        supported = ", ".join(f"'{k}'" for k in sorted(_REGISTRY))
        raise ValueError(f"Unknown protocol type: '{protocol_type}'. Supported types: {supported}")
    return ctor(num_agents, topology, config or {})
