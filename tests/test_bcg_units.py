"""Unit tests of the simulation layer (rules from SURVEY.md §2.4)."""
import os
import random

import pytest

from byzantine_consensus_llm_agents_amd.bcg.a2a_sim import A2AMessage, A2ASimProtocol, Decision, Phase
from byzantine_consensus_llm_agents_amd.bcg.agent_network import AgentNetwork, NetworkTopology
from byzantine_consensus_llm_agents_amd.bcg.byzantine_consensus import ByzantineConsensusGame
from byzantine_consensus_llm_agents_amd.bcg.protocol_factory import create_protocol


def test_topologies():
    fc = NetworkTopology.fully_connected(4)
    assert fc.adjacency_list[0] == [1, 2, 3]
    ring = NetworkTopology.ring(5)
    assert ring.adjacency_list[0] == [4, 1]
    grid = NetworkTopology.grid(2, 3)
    assert grid.num_agents == 6 and grid.adjacency_list[0] == [3, 1] and grid.adjacency_list[4] == [1, 3, 5]
    assert NetworkTopology.custom({0: [1], 1: [0]}).topology_type == "custom"


def test_a2a_ordering_dedupe_and_neighbors():
    proto = A2ASimProtocol(3, NetworkTopology.ring(3).adjacency_list)
    c2, c1 = proto.create_client(2), proto.create_client(1)
    c2.send_to_neighbors(1, Phase.PROPOSE.value, Decision("value", 5), "x" * 600)
    c1.send_to_neighbors(1, Phase.PROPOSE.value, Decision("value", 7), "hi")
    inbox = proto.deliver_messages(0, 1)
    assert [m.sender_id for m in inbox] == [1, 2]
    assert len(inbox[1].reasoning) == 500 and inbox[1].reasoning.endswith("...")
    dup = A2AMessage(1, 0, 1, "propose", Decision("value", 7), "other", 1)
    proto.send_message(1, 0, dup)  # same key -> suppressed
    assert proto.get_message_count(1) == 4
    with pytest.raises(ValueError):
        proto.send_message(0, 0, A2AMessage(0, 0, 1, "propose", Decision("value", 1), "", 9))
    msg = inbox[0]
    assert A2AMessage.from_dict(msg.to_dict()) == msg


def test_protocol_factory_unknown():
    with pytest.raises(ValueError, match="Unknown protocol type"):
        create_protocol("gossip", 2, {0: [1], 1: [0]})


def test_network_stats_off_by_one():
    topo = NetworkTopology.fully_connected(3)
    net = AgentNetwork(topo, create_protocol("a2a_sim", 3, topo.adjacency_list))
    for i in range(3):
        net.register_agent(f"agent_{i}", object(), i)
    for i in range(3):
        net.broadcast_message(f"agent_{i}", 0, Phase.PROPOSE, Decision("value", i), "r")
    assert net.get_network_stats()["total_messages"] == 0  # round 0 not counted yet
    net.advance_round()
    assert net.get_network_stats()["total_messages"] == 6


def _game(values, byz=()):
    g = ByzantineConsensusGame(num_honest=len(values) - len(byz), num_byzantine=len(byz),
                               value_range=(0, 50), max_rounds=3, rng=random.Random(0))
    for i, v in enumerate(values):
        st = g.agents[f"agent_{i}"]
        st.is_byzantine = i in byz
        st.initial_value = None if i in byz else v
        st.current_value = st.proposed_value = v
    return g


def test_consensus_rules():
    g = _game([3, 3, 3])
    assert g.check_consensus() == (True, 100.0)
    g = _game([3, 3, 4])
    ok, pct = g.check_consensus()
    assert not ok and abs(pct - 200 / 3) < 1e-9
    g = _game([3, 3, 9], byz=(2,))
    assert g.check_consensus() == (True, 100.0)
    g = _game([3, 4])
    for a in g.agents.values():
        a.current_value = 7  # unanimous on a non-initial value
    assert g.check_consensus() == (False, 100.0)


def test_termination_two_thirds_counts_abstainers():
    g = _game([1, 1, 1])
    assert g.should_terminate_by_vote({"agent_0": True, "agent_1": True, "agent_2": None})
    assert not g.should_terminate_by_vote({"agent_0": True, "agent_1": None, "agent_2": None})
    g.advance_round({"agent_0": True, "agent_1": True, "agent_2": False})
    assert g.game_over and g.termination_reason == "vote_with_consensus" and g.honest_agents_won
    st = g.get_statistics()
    assert st["consensus_outcome"] == "valid" and st["first_half_stop_reached"]


def test_deadline():
    g = _game([1, 2])
    for _ in range(3):
        g.advance_round({"agent_0": False, "agent_1": False})
    assert g.game_over and g.current_round == 4 and g.termination_reason == "max_rounds"
    assert g.get_statistics()["consensus_outcome"] == "timeout"


def test_reference_layout_shims_run_both_ways(tmp_path):
    """`cd byzantine_consensus_game; python main.py` (the reference workflow) and `python -m ...main`."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    args = ["--honest", "3", "--byzantine", "1", "--rounds", "2", "--engine", "fake", "--seed", "2"]
    env = dict(os.environ, PYTHONPATH=root)
    a = subprocess.run([sys.executable, os.path.join(root, "byzantine_consensus_game", "main.py"), *args],
                       cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert a.returncode == 0, a.stderr
    b = subprocess.run([sys.executable, "-m", "byzantine_consensus_game.main", *args], cwd=tmp_path, env=env,
                       capture_output=True, text=True, timeout=300)
    assert b.returncode == 0, b.stderr
    assert os.path.exists(tmp_path / "results" / "json" / "run_001.json")
    assert os.path.exists(tmp_path / "results" / "json" / "run_002.json")  # run numbers keep increasing
