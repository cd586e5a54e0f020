"""Topologies and the network facade over a communication protocol.

Parity target: reference ``bcg/agent_network.py`` (``NetworkTopology`` :12-87,
``AgentNetwork`` :90-237).  ``get_network_stats`` keeps the reference's
off-by-one (it sums message counts over ``range(current_round)``, so the last
round is only counted once the network has advanced past it).
"""

from dataclasses import dataclass
from typing import Any, Dict, List, Optional

from .a2a_sim import Decision, Phase
from .communication_protocol import CommunicationProtocol, Message, ProtocolClient


@dataclass
class NetworkTopology:
    """Static communication graph as an adjacency list."""

    num_agents: int
    adjacency_list: Dict[int, List[int]]
    topology_type: str

    @classmethod
    def fully_connected(cls, num_agents: int) -> "NetworkTopology":
        adj = {i: [j for j in range(num_agents) if j != i] for i in range(num_agents)}
        return cls(num_agents, adj, "fully_connected")

    @classmethod
    def ring(cls, num_agents: int) -> "NetworkTopology":
        adj = {i: [(i - 1) % num_agents, (i + 1) % num_agents] for i in range(num_agents)}
        return cls(num_agents, adj, "ring")

    @classmethod
    def grid(cls, rows: int, cols: int) -> "NetworkTopology":
        adj: Dict[int, List[int]] = {}
        for r in range(rows):
            for c in range(cols):
                nbrs = []
                # neighbour order: up, down, left, right
                for dr, dc in ((-1, 0), (1, 0), (0, -1), (0, 1)):
                    rr, cc = r + dr, c + dc
                    if 0 <= rr < rows and 0 <= cc < cols:
                        nbrs.append(rr * cols + cc)
                adj[r * cols + c] = nbrs
        return cls(rows * cols, adj, "grid")

    @classmethod
    def custom(cls, adjacency_list: Dict[int, List[int]]) -> "NetworkTopology":
        return cls(len(adjacency_list), adjacency_list, "custom")


class AgentNetwork:
    """Maps string agent ids onto protocol indices and forwards traffic."""

    def __init__(self, topology: NetworkTopology, protocol: CommunicationProtocol,
                 agents: Optional[Dict[str, Any]] = None):
        self.topology = topology
        self.num_agents = topology.num_agents
        self.protocol = protocol
        self.agents: Dict[str, Any] = agents or {}
        self.agent_id_to_index: Dict[str, int] = {}
        self.index_to_agent_id: Dict[int, str] = {}
        self.clients: Dict[str, ProtocolClient] = {}
        self.current_round = 0
        self.message_history: List[Message] = []

    def register_agent(self, agent_id: str, agent: Any, agent_index: int):
        self.agents[agent_id] = agent
        self.agent_id_to_index[agent_id] = agent_index
        self.index_to_agent_id[agent_index] = agent_id
        client = self.protocol.create_client(agent_index)
        self.clients[agent_id] = client
        setter = getattr(agent, "set_a2a_client", None)
        if setter is not None:
            setter(client)

    def broadcast_message(self, sender_id: str, round_num: int, phase: Phase,
                          decision: Decision, reasoning: str):
        self.clients[sender_id].send_to_neighbors(
            round=round_num, phase=phase.value, decision=decision, reasoning=reasoning)

    def get_messages(self, receiver_id: str, round_num: int, phase: Phase) -> List[Message]:
        return self.clients[receiver_id].receive_messages(round=round_num)

    def advance_round(self):
        self.current_round += 1

    def get_conversation_history(self, agent_id: str,
                                 max_messages: Optional[int] = None) -> List[Dict[str, Any]]:
        history = self.clients[agent_id].get_history()
        return history[-max_messages:] if max_messages else history

    def get_network_stats(self) -> Dict[str, Any]:
        counted = range(self.current_round)  # reference off-by-one preserved
        degree_sum = sum(len(n) for n in self.topology.adjacency_list.values())
        return {
            "num_agents": self.num_agents,
            "topology_type": self.topology.topology_type,
            "current_round": self.current_round,
            "total_messages": sum(self.protocol.get_message_count(r) for r in counted),
            "avg_degree": degree_sum / self.num_agents,
        }
