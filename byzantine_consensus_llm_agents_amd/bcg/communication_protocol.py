"""Pluggable communication-protocol interfaces.

Behavioural parity with the reference ABCs (``bcg/communication_protocol.py:14-217``):
``Message`` (serialisable, hashable for duplicate suppression), ``ProtocolClient``
(one per agent) and ``CommunicationProtocol`` (routing + delivery, with an
optional ``get_message_count`` that defaults to 0).
"""

from abc import ABC, abstractmethod
from dataclasses import dataclass
from typing import Any, Dict, List


@dataclass
class Message(ABC):
    """Base message: every protocol message carries sender, receiver and round."""

    sender_id: int
    receiver_id: int
    round: int

    @abstractmethod
    def to_dict(self) -> Dict[str, Any]:
        """JSON-compatible serialisation."""

    @classmethod
    @abstractmethod
    def from_dict(cls, data: Dict[str, Any]) -> "Message":
        """Inverse of :meth:`to_dict`."""

    @abstractmethod
    def __hash__(self):
        """Identity used for duplicate suppression."""

    @abstractmethod
    def __eq__(self, other):
        """Equality used for duplicate suppression."""


class ProtocolClient(ABC):
    """Per-agent handle onto a protocol instance."""

    def __init__(self, agent_id: int, protocol: "CommunicationProtocol"):
        self.agent_id = agent_id
        self.protocol = protocol

    @abstractmethod
    def receive_messages(self, round: int) -> List[Message]:
        """Inbox for ``round``."""

    @abstractmethod
    def send_to_neighbors(self, round: int, **kwargs):
        """Multicast a message to every neighbour."""

    @abstractmethod
    def get_neighbors(self) -> List[int]:
        """Neighbour indices of this client's agent."""

    @abstractmethod
    def get_history(self) -> List[Dict[str, Any]]:
        """Persistent per-agent communication history."""

    @abstractmethod
    def reset(self):
        """Clear client state for a fresh run."""


class CommunicationProtocol(ABC):
    """Routing + delivery over a static adjacency list."""

    def __init__(self, num_agents: int, topology: Dict[int, List[int]]):
        self.num_agents = num_agents
        self.topology = topology

    @abstractmethod
    def create_client(self, agent_id: int) -> ProtocolClient:
        """Factory for the agent-side client."""

    @abstractmethod
    def send_message(self, sender_id: int, receiver_id: int, message: Message):
        """Point-to-point send."""

    @abstractmethod
    def deliver_messages(self, agent_id: int, round: int) -> List[Message]:
        """All messages addressed to ``agent_id`` in ``round``."""

    @abstractmethod
    def get_neighbors(self, agent_id: int) -> List[int]:
        """Neighbour indices of ``agent_id``."""

    @abstractmethod
    def reset(self):
        """Clear protocol state for a fresh run."""

    def get_message_count(self, round: int) -> int:
        """Messages buffered for ``round`` (metrics only; optional)."""
        return 0
