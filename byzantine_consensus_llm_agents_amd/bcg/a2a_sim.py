"""A2A-Sim: synchronous, lossless, in-memory agent-to-agent message bus.

Parity target: reference ``bcg/a2a_sim.py`` (Phase/DecisionType enums :20-32,
Decision :35-46, A2AMessage :49-113, A2ASimProtocol :116-298,
A2ASimClient :301-387).  Semantics preserved:

* messages are buffered per ``round -> receiver -> [msg]`` and only neighbours
  may be addressed (``ValueError`` otherwise);
* duplicates are suppressed on ``(sender, receiver, round, phase, timestamp)``;
* inboxes are returned ordered by ``(sender_id, timestamp)``;
* reasoning longer than 500 characters is cut to 497 + ``"..."``;
* every client owns a monotonically increasing timestamp counter.

The bus stays pure Python on purpose: it moves O(N^2) tiny objects per round,
which is noise next to one batched LLM pass on the GPU.
"""

from dataclasses import dataclass
from enum import Enum
from typing import Any, Dict, List, Set

from .communication_protocol import CommunicationProtocol, Message, ProtocolClient

REASONING_LIMIT = 500


class Phase(str, Enum):
    PROPOSE = "propose"
    PREPARE = "prepare"
    COMMIT = "commit"
    CUSTOM = "custom"


class DecisionType(str, Enum):
    VALUE = "value"
    VOTE = "vote"
    ABSTAIN = "abstain"


@dataclass
class Decision:
    """Machine-readable half of an A2A message."""

    type: str
    value: Any

    def to_dict(self) -> Dict[str, Any]:
        return {"type": self.type, "value": self.value}

    @classmethod
    def from_dict(cls, data: Dict[str, Any]) -> "Decision":
        return cls(type=data["type"], value=data["value"])


def _clip_reasoning(text: str) -> str:
    if len(text) <= REASONING_LIMIT:
        return text
    return text[: REASONING_LIMIT - 3] + "..."


@dataclass
class A2AMessage(Message):
    """Dual-payload message: structured decision + natural-language reasoning."""

    sender_id: int
    receiver_id: int
    round: int
    phase: str
    decision: Decision
    reasoning: str
    timestamp: int

    def __post_init__(self):
        self.reasoning = _clip_reasoning(self.reasoning)

    def _key(self):
        return (self.sender_id, self.receiver_id, self.round, self.phase, self.timestamp)

    def to_dict(self) -> Dict[str, Any]:
        out = {
            "sender_id": self.sender_id,
            "receiver_id": self.receiver_id,
            "round": self.round,
            "phase": self.phase,
        }
        out["decision"] = self.decision.to_dict()
        out["reasoning"] = self.reasoning
        out["timestamp"] = self.timestamp
        return out

    @classmethod
    def from_dict(cls, data: Dict[str, Any]) -> "A2AMessage":
        fields = dict(data)
        fields["decision"] = Decision.from_dict(data["decision"])
        return cls(**{k: fields[k] for k in
                      ("sender_id", "receiver_id", "round", "phase", "decision",
                       "reasoning", "timestamp")})

    def __hash__(self):
        return hash(self._key())

    def __eq__(self, other):
        return isinstance(other, A2AMessage) and self._key() == other._key()


class A2ASimProtocol(CommunicationProtocol):
    """Router over a static graph G=(V,E) given as an adjacency list."""

    def __init__(self, num_agents: int, topology: Dict[int, List[int]]):
        super().__init__(num_agents, topology)
        self.message_buffer: Dict[int, Dict[int, List[A2AMessage]]] = {}
        self.delivered: Set[A2AMessage] = set()
        self.current_round = 0
        self.current_phase = Phase.PROPOSE.value

    # -- routing ------------------------------------------------------------
    def send_message(self, sender_id: int, receiver_id: int, message: A2AMessage):
        if receiver_id not in self.topology.get(sender_id, []):
            raise ValueError(
                f"Agent {sender_id} cannot send to {receiver_id}: not in neighbor set")
        if message in self.delivered:
            return
        self.message_buffer.setdefault(message.round, {}).setdefault(receiver_id, []).append(message)
        self.delivered.add(message)

    def broadcast_to_neighbors(self, sender_id: int, round: int, phase: str,
                               decision: Decision, reasoning: str, timestamp: int):
        """Send the same payload to every neighbour of ``sender_id``."""
        for receiver in self.topology.get(sender_id, []):
            self.send_message(sender_id, receiver, A2AMessage(
                sender_id, receiver, round, phase, decision, reasoning, timestamp))

    def deliver_messages(self, agent_id: int, round: int) -> List[A2AMessage]:
        inbox = self.message_buffer.get(round, {}).get(agent_id, [])
        return sorted(inbox, key=lambda m: (m.sender_id, m.timestamp))

    # -- bookkeeping --------------------------------------------------------
    def clear_round_buffer(self, round: int):
        self.message_buffer.pop(round, None)

    def get_neighbors(self, agent_id: int) -> List[int]:
        return self.topology.get(agent_id, [])

    def set_phase(self, round: int, phase: str):
        self.current_round = round
        self.current_phase = phase

    def get_message_count(self, round: int) -> int:
        return sum(len(v) for v in self.message_buffer.get(round, {}).values())

    def reset(self):
        self.message_buffer.clear()
        self.delivered.clear()
        self.current_round = 0

    def create_client(self, agent_id: int) -> "A2ASimClient":
        return A2ASimClient(agent_id=agent_id, protocol=self)


class A2ASimClient(ProtocolClient):
    """Agent-side view: send to neighbours, read inbox, keep history H_i."""

    def __init__(self, agent_id: int, protocol: A2ASimProtocol):
        super().__init__(agent_id, protocol)
        self.protocol: A2ASimProtocol = protocol
        self.history: List[Dict[str, Any]] = []
        self._timestamp_counter = 0

    def next_timestamp(self) -> int:
        self._timestamp_counter += 1
        return self._timestamp_counter

    def receive_messages(self, round: int) -> List[A2AMessage]:
        return self.protocol.deliver_messages(self.agent_id, round)

    def send_to_neighbors(self, round: int, phase: str, decision: Decision, reasoning: str):
        self.protocol.broadcast_to_neighbors(self.agent_id, round, phase, decision,
                                             reasoning, self.next_timestamp())

    def update_history(self, round: int, inbox: List[A2AMessage], local_state: Dict[str, Any]):
        self.history.append({"round": round,
                             "inbox": [m.to_dict() for m in inbox],
                             "local_state": local_state})

    def get_neighbors(self) -> List[int]:
        return self.protocol.get_neighbors(self.agent_id)

    def get_history(self) -> List[Dict[str, Any]]:
        return self.history

    def reset(self):
        self.history.clear()
        self._timestamp_counter = 0
