"""BCG simulator: round loop, batched decide/vote with retry ladder, persistence.

Parity target: reference ``bcg/main.py`` ``BCGSimulation`` (:67-995).

Round structure (reference ``run_round`` :517-658):
  decide (one batched engine call, retries) -> broadcast over A2A-sim ->
  receive (agent.my_value <- proposed value) -> round summaries ->
  store reasoning -> vote (one batched call, retries) -> game.advance_round ->
  network.advance_round.

Retry ladder (reference :256-478): after a batch attempt,
if the failed fraction is <= 30% and attempts remain, the failed agents run
their own sequential 3-attempt path and the ladder stops; otherwise the failed
subset is re-batched (max 3 batch attempts).  Failed decides abstain, failed
votes default to continue.  A Byzantine "abstain" vote is *invalid* for the
batched validator and is therefore always re-asked sequentially (quirk kept).

Additions over the reference (all opt-in, defaults unchanged):
  * ``config["seed"]`` gives the game its own ``random.Random`` so several
    simulations can share a process (DP packing) deterministically;
  * per-simulation counters (``self.counters``) of accepted decisions and
    engine calls, used by the decisions/sec benchmark.
"""

import csv
import json
import os
import random
import threading
from datetime import datetime
from typing import Dict, List, Optional, Tuple

from . import bcg_agents
from .a2a_sim import Decision, DecisionType, Phase
from .agent_network import AgentNetwork, NetworkTopology
from .bcg_agents import create_agent
from .byzantine_consensus import ByzantineConsensusGame
from .config import (AGENT_CONFIG, BCG_CONFIG, COMMUNICATION_CONFIG, LLM_CONFIG, METRICS_CONFIG,
                     NETWORK_CONFIG, VLLM_CONFIG)
from .protocol_factory import create_protocol

MAX_RETRIES = 3
BATCH_RETRY_THRESHOLD = 0.3

_log_file = None

CSV_FIELDS = [
    "run_number", "timestamp",
    "consensus_reached", "consensus_outcome", "honest_agents_won", "total_rounds", "max_rounds",
    "consensus_value",
    "convergence_speed", "consensus_is_median", "consensus_is_extreme", "consensus_is_initial",
    "trajectory_stability", "final_convergence_metric", "convergence_rate_percent",
    "centrality", "inclusivity", "stability_rounds", "agreement_rate", "consensus_quality_score",
    "avg_distance_from_consensus", "byzantine_infiltration",
    "honest_initial_mean", "honest_initial_median", "honest_initial_std", "honest_final_std",
    "a2a_message_count",
    "value_range", "network_topology", "model_name", "byzantine_strategy", "honest_agent_type",
    "protocol_type",
]

CSV_PRECISION = {
    "final_convergence_metric": 1, "convergence_rate_percent": 1, "agreement_rate": 1,
    "consensus_quality_score": 1, "avg_distance_from_consensus": 3, "honest_initial_std": 3,
    "honest_final_std": 3, "byzantine_infiltration": 1, "centrality": 3, "inclusivity": 3,
    "trajectory_stability": 3, "honest_initial_mean": 2, "honest_initial_median": 2,
}


def tee_print(*args, **kwargs):
    print(*args, **kwargs)
    if _log_file:
        print(*args, **kwargs, file=_log_file, flush=True)


def _next_run_number(json_dir: str) -> int:
    nums = []
    for name in os.listdir(json_dir):
        if name.startswith("run_") and name.endswith(".json"):
            try:
                nums.append(int(name[4:-5]))
            except ValueError:
                pass
    return max(nums) + 1 if nums else 1


def _vote_label(vote) -> str:
    return "STOP" if vote is True else ("CONTINUE" if vote is False else "ABSTAIN")


def is_valid_decision(result: Optional[Dict]) -> bool:
    """Batched-path validity (reference :232-247)."""
    if result is None or "error" in result or result.get("value") is None:
        return False
    internal = result.get("internal_strategy", "")
    reasoning = result.get("public_reasoning", "")
    return (isinstance(internal, str) and len(internal.strip()) >= 3
            and isinstance(reasoning, str) and len(reasoning.strip()) >= 10)


def is_valid_vote(result: Optional[Dict]) -> bool:
    """Batched-path validity (reference :249-254): abstain is NOT accepted here."""
    if result is None or "error" in result:
        return False
    return result.get("decision", "") in ["stop", "continue"]


def run_concurrently(engine_agent, jobs):
    """Run independent per-agent retry ladders concurrently (one engine batch per attempt).

    The reference runs them one agent after another (main.py:327-333,
    :432-437); each ladder only depends on its own agent, so running them in
    threads whose engine calls the LLM coalesces yields the same per-agent
    results with one engine call per attempt instead of one per agent.
    """
    llm = getattr(engine_agent, "llm", None)
    if len(jobs) <= 1 or llm is None or not hasattr(llm, "register_client"):
        return [job() for job in jobs]
    results = [None] * len(jobs)
    errors = []

    parent_key = getattr(threading.current_thread(), "_bcg_order_key", ())

    def work(i, job):
        threading.current_thread()._bcg_order_key = tuple(parent_key) + (i,)
        try:
            results[i] = job()
        except BaseException as exc:
            errors.append(exc)
        finally:
            llm.unregister_client()

    for _ in range(len(jobs)):
        llm.register_client()
    threads = [threading.Thread(target=work, args=(i, j)) for i, j in enumerate(jobs)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errors:
        raise errors[0]
    return results


def topology_for(num_agents: int) -> NetworkTopology:
    kind = NETWORK_CONFIG["topology_type"]
    if kind == "ring":
        return NetworkTopology.ring(num_agents)
    if kind == "custom":
        return NetworkTopology.custom(NETWORK_CONFIG["custom_adjacency"])
    return NetworkTopology.fully_connected(num_agents)  # also the fallback for 'grid'


class BCGSimulation:
    """One Byzantine Consensus Game with LLM agents on an A2A-sim network."""

    def __init__(self, num_honest: int = 7, num_byzantine: int = 3, config: dict = None):
        global _log_file
        self.config = {**BCG_CONFIG, **(config or {})}
        self.config["num_honest"] = num_honest
        self.config["num_byzantine"] = num_byzantine
        self.log_buffer: List[str] = []
        self.verbose = config.get("verbose", False) if config else False
        self._log_file = None
        # accepted outputs (the headline metric) and the retry ladder's cost: engine calls,
        # rows sent to batch calls (first attempts + re-batched failures), sequential
        # re-queries, and outputs that exhausted every attempt (abstain / default CONTINUE)
        self.counters = {"decisions_accepted": 0, "votes_accepted": 0,
                         "decide_batches": 0, "vote_batches": 0, "sequential_calls": 0,
                         "decide_prompts": 0, "vote_prompts": 0, "batch_rows": 0,
                         "sequential_attempts": 0, "decisions_exhausted": 0, "votes_exhausted": 0}

        json_dir = os.path.join(METRICS_CONFIG["results_dir"], "json")
        if METRICS_CONFIG.get("save_results", True):
            os.makedirs(json_dir, exist_ok=True)
            self.run_number = f"{_next_run_number(json_dir):03d}"
            log_dir = os.path.join(METRICS_CONFIG["results_dir"], "logs")
            os.makedirs(log_dir, exist_ok=True)
            log_path = os.path.join(log_dir, f"run_{self.run_number}_log.txt")
            _log_file = open(log_path, "w", buffering=1)
            self._log_file = _log_file
            tee_print(f"Starting run {self.run_number} - Logging to: {log_path}")
        else:
            # no results dir is created when nothing will be saved
            self.run_number = (f"{_next_run_number(json_dir):03d}" if os.path.isdir(json_dir) else "001")
            _log_file = None
        bcg_agents.set_agent_log_file(self._log_file)

        seed = self.config.get("seed")
        rng = random.Random(seed) if seed is not None else None
        self.game = ByzantineConsensusGame(
            num_honest=num_honest, num_byzantine=num_byzantine,
            value_range=self.config["value_range"],
            consensus_threshold=self.config["consensus_threshold"],
            max_rounds=self.config["max_rounds"], rng=rng)

        n = num_honest + num_byzantine
        topo = topology_for(n)
        protocol = create_protocol(COMMUNICATION_CONFIG["protocol_type"], n,
                                   topo.adjacency_list, COMMUNICATION_CONFIG)
        self.network = AgentNetwork(topo, protocol=protocol)
        self.agents: Dict[str, bcg_agents.BCGAgent] = {}
        self._create_agents()

    # --------------------------------------------------------------- logging
    def log(self, message: str, level: str = "INFO"):
        line = f"[{level}] {message}"
        self.log_buffer.append(line)
        if self._log_file:
            self._log_file.write(line + "\n")
            self._log_file.flush()
        if self.verbose:
            print(message)

    # ----------------------------------------------------------------- setup
    def _create_agents(self):
        self.log("\n" + "=" * 60)
        self.log("Creating agents...")
        self.log(f"Model: {VLLM_CONFIG['model_name']}")
        self.log(f"Quantization: {VLLM_CONFIG.get('quantization', 'None (full precision)')}")
        self.log("=" * 60)
        value_range = BCG_CONFIG.get("value_range", (0, 50))  # global, as in the reference
        awareness = self.config.get("byzantine_awareness", "may_exist")
        self.log(f"Byzantine awareness: {awareness}")
        for idx, agent_id in enumerate(sorted(self.game.agents)):  # lexicographic order
            game_state = self.game.agents[agent_id]
            self.log(f"\nCreating agent: {agent_id}")
            agent = create_agent(agent_id=agent_id, is_byzantine=game_state.is_byzantine,
                                 model_name=VLLM_CONFIG["model_name"], model_config=VLLM_CONFIG,
                                 value_range=value_range, byzantine_awareness=awareness)
            if game_state.initial_value is not None:
                agent.set_initial_value(game_state.initial_value)
            self.network.register_agent(agent_id, agent, idx)
            self.agents[agent_id] = agent
        self.log("\n" + "=" * 60)
        self.log(f"All agents created! Total: {len(self.agents)}")
        self.log("=" * 60 + "\n")

    def _engine_agent(self):
        return next(iter(self.agents.values()))

    def _is_valid_decision_response(self, result: Dict) -> bool:
        return is_valid_decision(result)

    def _is_valid_vote_response(self, result: Dict) -> bool:
        return is_valid_vote(result)

    # ------------------------------------------------------- retry ladder
    def _attempts(self, pending) -> int:
        """Engine calls the agents' own sequential retry loops have made so far."""
        return sum(getattr(self.agents[aid], "sequential_attempts", 0) for aid, _ in pending)

    def _ladder(self, jobs: List[Tuple[str, tuple]], temperature: float, max_tokens: int,
                valid, sequential, kind: str) -> Dict[str, Optional[Dict]]:
        """Shared batch-then-sequential retry policy for both phases."""
        results: Dict[str, Optional[Dict]] = {aid: None for aid, _ in jobs}
        if not jobs:
            return results
        engine = next(iter(self.agents.values()))
        self.counters["decide_prompts" if kind == "agents" else "vote_prompts"] += len(jobs)
        pending = list(jobs)
        for attempt in range(1, MAX_RETRIES + 1):
            if not pending:
                break
            if attempt == 1:
                self.log(f"  [BATCHED] Processing {len(pending)} {kind} in single LLM call...")
            else:
                self.log(f"  [RETRY {attempt}/{MAX_RETRIES}] Retrying {len(pending)} failed {kind}...")
            self.counters["decide_batches" if kind == "agents" else "vote_batches"] += 1
            self.counters["batch_rows"] += len(pending)
            outs = engine.batch_generate_json([p for _, p in pending], temperature=temperature,
                                              max_tokens=max_tokens)
            failed = []
            for (aid, prompt), res in zip(pending, outs):
                if valid(res):
                    results[aid] = res
                else:
                    failed.append((aid, prompt))
                    what = "response" if kind == "agents" else "vote"
                    self.log(f"  ⚠️ [{aid}] Invalid {what} on attempt {attempt}")
            pending = failed
            if pending and attempt < MAX_RETRIES and len(pending) / len(jobs) <= BATCH_RETRY_THRESHOLD:
                share = f" (<{BATCH_RETRY_THRESHOLD * 100:.0f}%)" if kind == "agents" else ""
                self.log(f"  [SEQUENTIAL RETRY] {len(pending)} {kind} failed{share}, retrying individually...")
                pending = sequential(pending, results)
                break
        return results

    def _run_batched_decisions(self, round_num: int, game_state: Dict):
        jobs = []
        for aid, agent in self.agents.items():
            prompt = agent.build_decision_prompt(game_state)
            if prompt is None:
                self.log(f"  {aid}: ERROR - no prompt returned")
            else:
                jobs.append((aid, prompt))
        if not jobs:
            return

        def sequential(pending, results):
            self.counters["sequential_calls"] += len(pending)
            before = self._attempts(pending)
            values = run_concurrently(self._engine_agent(), [
                (lambda a=self.agents[aid]: a.decide_next_value(game_state)) for aid, _ in pending])
            self.counters["sequential_attempts"] += self._attempts(pending) - before
            still = []
            for (aid, prompt), value in zip(pending, values):
                if value is not None:
                    results[aid] = {"_sequential_success": True, "value": value}
                else:
                    still.append((aid, prompt))
            return still

        results = self._ladder(jobs, LLM_CONFIG["temperature_decide"], LLM_CONFIG["max_tokens_decide"],
                               is_valid_decision, sequential, "agents")
        failed = [aid for aid, r in results.items() if r is None]
        if failed:
            self.log(f"  ❌ {len(failed)} agents failed all {MAX_RETRIES} attempts - they will abstain")

        for aid, _ in jobs:
            agent = self.agents[aid]
            res = results.get(aid)
            if res is None:
                self.counters["decisions_exhausted"] += 1
                agent.last_reasoning = f"⚠️ All {MAX_RETRIES} attempts failed - abstaining"
                self.log(f"  {aid}: ABSTAINING (all attempts failed)")
                continue
            self.counters["decisions_accepted"] += 1
            value = res.get("value") if res.get("_sequential_success") else agent.parse_decision_response(res, game_state)
            if value is None:
                self.log(f"  {aid}: ABSTAINING")
                self.log(f"    Reasoning: {getattr(agent, 'last_reasoning', '[abstaining]')}")
                continue
            value = int(round(value))
            self.game.update_agent_proposal(aid, value)
            before = f"{int(agent.my_value)}" if agent.my_value is not None else "(no value yet)"
            self.log(f"  {aid}: {before} -> {value}")
            self.log(f"    Reasoning: {getattr(agent, 'last_reasoning', 'No reasoning provided')}")

    def _run_batched_votes(self, game_state: Dict) -> Dict[str, Optional[bool]]:
        jobs = [(aid, agent.build_vote_prompt(game_state)) for aid, agent in self.agents.items()]

        def sequential(pending, results):
            self.counters["sequential_calls"] += len(pending)
            before = self._attempts(pending)
            votes = run_concurrently(self._engine_agent(), [
                (lambda a=self.agents[aid]: a.vote_to_terminate(game_state)) for aid, _ in pending])
            self.counters["sequential_attempts"] += self._attempts(pending) - before
            for (aid, _), vote in zip(pending, votes):
                results[aid] = {"_sequential_success": True, "vote": vote,
                                "_valid": getattr(self.agents[aid], "last_vote_valid", True)}
            return []

        results = self._ladder(jobs, LLM_CONFIG["temperature_vote"], LLM_CONFIG["max_tokens_vote"],
                               is_valid_vote, sequential, "votes")
        failed = [aid for aid, r in results.items() if r is None]
        if failed:
            self.log(f"  ❌ {len(failed)} votes failed all attempts - defaulting to CONTINUE")

        votes: Dict[str, Optional[bool]] = {}
        for aid, _ in jobs:
            res = results.get(aid)
            if res is None:
                self.counters["votes_exhausted"] += 1
                vote = False
                self.log(f"  {aid}: votes CONTINUE (default - all attempts failed)")
            else:
                # a sequential vote that exhausted its attempts is the game's default CONTINUE:
                # the game sees it exactly as the reference does, the counter does not
                if res.get("_valid", True):
                    self.counters["votes_accepted"] += 1
                else:
                    self.counters["votes_exhausted"] += 1
                if res.get("_sequential_success"):
                    vote = res.get("vote", False)
                else:
                    vote = self.agents[aid].parse_vote_response(res, game_state)
                self.log(f"  {aid}: votes {_vote_label(vote)}")
            votes[aid] = vote
        return votes

    def _update_round_summaries(self, round_num: int):
        parts = []
        for aid, agent in sorted(self.agents.items()):
            reasoning = getattr(agent, "last_reasoning", "")
            if reasoning and len(reasoning) > 50:
                reasoning = reasoning[:47] + "..."
            shown = "ABSTAINED" if agent.my_value is None else f"{int(agent.my_value)}"
            part = f"{aid} value: {shown}"
            if reasoning:
                part += f" | Reasoning: {reasoning}"
            parts.append(part)
        summary = f"Round {round_num}: " + "; ".join(parts)
        for agent in self.agents.values():
            agent.state.add_round_summary(summary, max_history=15)

    # -------------------------------------------------------------- rounds
    def _batched_enabled(self) -> bool:
        return (self.config.get("use_batched_inference", True)
                and AGENT_CONFIG.get("use_structured_output", False))

    def _decide_phase(self, round_num: int, game_state: Dict):
        if self._batched_enabled():
            self._run_batched_decisions(round_num, game_state)
            return
        for aid, agent in self.agents.items():
            value = agent.decide_next_value(game_state)
            if value is None:
                self.log(f"  {aid}: ABSTAINING")
                self.log(f"    Reasoning: {getattr(agent, 'last_reasoning', '[abstaining]')}")
                continue
            value = int(round(value))
            self.game.update_agent_proposal(aid, value)
            before = str(int(agent.my_value)) if agent.my_value is not None else "(none)"
            self.log(f"  {aid}: {before} -> {value}")
            self.log(f"    Reasoning: {getattr(agent, 'last_reasoning', 'No reasoning provided')}")

    def _vote_phase(self, game_state: Dict) -> Dict[str, Optional[bool]]:
        if self._batched_enabled():
            return self._run_batched_votes(game_state)
        votes = {}
        for aid, agent in self.agents.items():
            votes[aid] = agent.vote_to_terminate(game_state)
            self.log(f"  {aid}: votes {_vote_label(votes[aid])}")
        return votes

    def run_round(self):
        round_num = self.game.current_round
        self.log(f"\n{'=' * 60}")
        self.log(f"Round {round_num}")
        self.log(f"{'=' * 60}")
        phase = Phase.PROPOSE
        game_state = self.game.get_game_state()

        self.log("\n[Decision Phase - LLM Reasoning]")
        self._decide_phase(round_num, game_state)

        self.log("\n[Broadcast Phase]")
        for aid, agent in self.agents.items():
            proposed = self.game.agents[aid].proposed_value
            if proposed is None:
                self.log(f"  {aid}: (abstaining, no broadcast)")
                continue
            reasoning = getattr(agent, "last_reasoning", f"Proposing value: {int(proposed)}")
            self.network.broadcast_message(
                sender_id=aid, round_num=round_num, phase=phase,
                decision=Decision(type=DecisionType.VALUE.value, value=int(proposed)),
                reasoning=reasoning)
            tag = " (Byzantine)" if getattr(agent, "is_byzantine", False) else ""
            self.log(f"  {aid}{tag}: broadcasts value {int(proposed)}")

        self.log("\n[Receive Phase - Updating State]")
        for aid, agent in self.agents.items():
            inbox = self.network.get_messages(aid, round_num, phase)
            proposals = [(self.network.index_to_agent_id[m.sender_id], m.decision.value, m.reasoning)
                         for m in inbox]
            agent.receive_proposals(proposals)
            agent.my_value = self.game.agents[aid].proposed_value
            self.log(f"  {aid}: received {len(proposals)} proposals, updated state")

        self._update_round_summaries(round_num)
        self.game.store_round_reasoning({aid: a.last_reasoning for aid, a in self.agents.items()
                                         if getattr(a, "last_reasoning", "")})

        self.log("\n[Voting Phase]")
        votes = self._vote_phase(game_state)  # NB: round-start snapshot, as in the reference
        info = self.game.get_all_termination_votes(votes)
        self.log(f"\n  All agents voting to stop: {info['total_stop_votes']}/{info['total_agents']}")
        self.log(f"    (Honest: {info['honest_stop_votes']}, Byzantine: {info['byzantine_stop_votes']})")

        self.game.advance_round(votes)
        self.network.advance_round()
        last = self.game.rounds[-1]
        self.log(f"\n[Round {round_num} Summary]")
        self.log(f"  Most common value: {last.consensus_value}")
        self.log(f"  Agreement: {last.agreement_count}/{self.config['num_honest']} honest agents "
                 f"({last.convergence_metric:.1f}%)")
        self.log(f"  Consensus reached: {last.has_consensus}")

    def run(self):
        self.log("\n" + "=" * 60)
        self.log("BYZANTINE CONSENSUS GAME - Simulation Started")
        self.log("=" * 60)
        self.log("\n[Initial State]")
        self.log(f"  Total agents: {self.config['num_honest'] + self.config['num_byzantine']}")
        self.log(f"  Honest agents: {self.config['num_honest']}")
        self.log(f"  Byzantine agents: {self.config['num_byzantine']} (hidden)")
        self.log("  Consensus requires: 66% agreement (supermajority)")
        self.log(f"  Max rounds: {self.config['max_rounds']}")
        self.log("\n[Initial Values]")
        for aid, st in self.game.agents.items():
            shown = int(st.initial_value) if st.initial_value is not None else "(no initial value)"
            self.log(f"  {aid}: {shown}")
        while not self.game.game_over:
            self.run_round()
        self.display_results()
        if METRICS_CONFIG["save_results"]:
            self.save_results()

    # ------------------------------------------------------------ reporting
    def display_results(self):
        self.log("\n" + "=" * 60)
        self.log("SIMULATION COMPLETE")
        self.log("=" * 60)
        s = self.game.get_statistics()
        self.log("\n[Final Results]")
        self.log(f"  Total rounds: {s['total_rounds']}")
        self.log(f"  Max rounds (deadline): {s['max_rounds']}")
        self.log(f"  Consensus reached: {s['consensus_reached']}")
        won = s["honest_agents_won"]
        self.log("  HONEST AGENTS WON - Consensus reached!" if won is True else
                 "  HONEST AGENTS LOST - No consensus achieved" if won is False else
                 "  Game ended without clear outcome")
        if s["consensus_reached"]:
            self.log(f"  Consensus value: {int(s['consensus_value'])}")
            self.log(f"  Agreement rate: {s['agreement_rate']:.1f}% of honest agents")
            self.log(f"  Avg distance from consensus: {s['avg_distance_from_consensus']:.2f}")
        self.log("\n[Honest Agents]")
        self.log(f"  Initial mean: {s['honest_initial_mean']:.1f} (±{s['honest_initial_std']:.2f})")
        self.log(f"  Final mean: {s['honest_final_mean']:.1f} (±{s['honest_final_std']:.2f})")
        if s["consensus_reached"]:
            q = s["consensus_quality_score"]
            self.log("\n[Consensus Quality Analysis]")
            self.log(f"  Consensus quality score: {q:.0f}/100")
            infil = s["byzantine_infiltration"]
            # the reference crashes here (None:.1f) when 0 Byzantine agents reach consensus
            infil_txt = f"{infil:.1f}%" if infil is not None else "n/a (no Byzantine agents)"
            self.log(f"  Byzantine infiltration: {infil_txt} voted for consensus")
            self.log("   Excellent - consensus close to honest agents' initial values" if q >= 90 else
                     "   Moderate - Byzantine agents had some influence" if q >= 70 else
                     "   Poor - Byzantine agents significantly pulled consensus away")
        self.log("\n[Final Values]")
        cval = int(s["consensus_value"]) if s["consensus_reached"] else None
        for aid, st in self.game.agents.items():
            final = int(st.current_value) if st.current_value is not None else "(none)"
            if st.initial_value is not None:
                initial = int(st.initial_value)
                delta = f"(Δ {final - initial:+d})" if isinstance(final, int) else ""
            else:
                initial, delta = "(none)", ""
            if cval is not None and isinstance(final, int) and final == cval:
                marker = " ⚠️ [BYZANTINE]" if st.is_byzantine else " ✓"
            else:
                marker = " [BYZANTINE]" if st.is_byzantine else ""
            print(f"  {aid}: {initial} -> {final} {delta}{marker}")
        print("\n[Byzantine Agents Revealed]")
        self.log(f"  Byzantine: {', '.join(a for a, st in self.game.agents.items() if st.is_byzantine)}")
        self.log(f"  Honest: {', '.join(a for a, st in self.game.agents.items() if not st.is_byzantine)}")
        if s["consensus_reached"]:
            self.log("\n[Network Evaluation]")
            ar, q = s["agreement_rate"], s["consensus_quality_score"]
            if ar >= 90 and q >= 85:
                print("  🎯 EXCELLENT: Network successfully converged to honest consensus")
            elif ar >= 70 and q >= 70:
                print("  ✓ GOOD: Network reached consensus with moderate quality")
            elif ar >= 50:
                print("  ⚠️  WEAK: Network barely reached consensus, quality low")
            else:
                print("  ✗ POOR: Network consensus unreliable")
        net = self.network.get_network_stats()
        self.log("\n[Communication Statistics]")
        self.log(f"  Total messages: {net['total_messages']}")
        per_round = net["total_messages"] // s["total_rounds"] if s["total_rounds"] > 0 else 0
        self.log(f"  Messages per round: {per_round}")
        self.log(f"  Topology: {net['topology_type']}")
        self.log(f"  Average degree: {net['avg_degree']:.1f}")

    def a2a_message_count(self) -> int:
        # reference quirk (main.py:804-807): range(current_round) omits the
        # final round after a stop-by-vote, includes it after the deadline
        return sum(self.network.protocol.get_message_count(r) for r in range(self.game.current_round))

    def results_payload(self) -> Dict:
        timestamp = datetime.now().strftime("%Y%m%d_%H%M%S")
        stats = self.game.get_statistics()
        count = self.a2a_message_count()
        metrics = self._build_metrics_payload(stats=stats, timestamp=timestamp, message_count=count)
        return {
            "run_number": int(self.run_number),
            "timestamp": timestamp,
            "config": self.config,
            "statistics": stats,
            "metrics": metrics,
            "rounds": [{"round": r.round_num, "honest_mean": r.honest_mean, "honest_std": r.honest_std,
                        "convergence_metric": r.convergence_metric, "has_consensus": r.has_consensus}
                       for r in self.game.rounds],
            "final_state": self.game.get_game_state(),
            "a2a_message_count": count,
        }

    def save_results(self):
        json_dir = os.path.join(METRICS_CONFIG["results_dir"], "json")
        os.makedirs(json_dir, exist_ok=True)
        path = os.path.join(json_dir, f"run_{self.run_number}.json")
        payload = self.results_payload()
        with open(path, "w") as fh:
            json.dump(payload, fh, indent=2)
        self._save_metrics_snapshot(payload["metrics"])
        self.log("\n[Results Saved]")
        self.log(f"  JSON: {path}")
        self.log(f"  Log: run_{self.run_number}.log (already saved)")
        print(f"Results: {path}")
        print(f"Metrics: {os.path.join(METRICS_CONFIG['results_dir'], 'metrics', f'run_{self.run_number}.csv')}")

    def _build_metrics_payload(self, stats: dict, timestamp: str, message_count: int) -> dict:
        g = stats.get
        rate = g("convergence_rate")
        vr = list(self.config.get("value_range", ()))
        m = {"run_number": int(self.run_number), "timestamp": timestamp}
        for key in ("consensus_reached", "consensus_outcome", "honest_agents_won", "total_rounds",
                    "max_rounds", "consensus_value", "convergence_speed", "consensus_is_median",
                    "consensus_is_extreme", "consensus_is_initial", "trajectory_stability",
                    "final_convergence_metric"):
            m[key] = g(key)
        m["convergence_rate_percent"] = rate * 100 if rate is not None else None
        for key in ("centrality", "inclusivity", "stability_rounds", "agreement_rate",
                    "consensus_quality_score", "avg_distance_from_consensus", "byzantine_infiltration",
                    "honest_initial_mean", "honest_initial_median", "honest_initial_std",
                    "honest_final_std"):
            m[key] = g(key)
        m["a2a_message_count"] = message_count
        m["value_range"] = vr if vr else None
        m["network_topology"] = NETWORK_CONFIG.get("topology_type")
        m["model_name"] = VLLM_CONFIG.get("model_name")
        m["byzantine_strategy"] = AGENT_CONFIG.get("byzantine_strategy")
        m["honest_agent_type"] = AGENT_CONFIG.get("honest_agent_type")
        m["protocol_type"] = COMMUNICATION_CONFIG.get("protocol_type")
        return m

    def _save_metrics_snapshot(self, metrics: dict):
        out_dir = os.path.join(METRICS_CONFIG["results_dir"], "metrics")
        os.makedirs(out_dir, exist_ok=True)
        path = os.path.join(out_dir, f"run_{self.run_number}.csv")
        row = {}
        for key in CSV_FIELDS:
            value = metrics.get(key)
            if key in CSV_PRECISION and value is not None:
                try:
                    value = round(float(value), CSV_PRECISION[key])
                except (TypeError, ValueError):
                    pass
            if value is None:
                value = ""
            elif isinstance(value, list):
                value = "-".join(str(v) for v in value)
            elif isinstance(value, bool):
                value = str(value)
            row[key] = value
        with open(path, "w", newline="") as fh:
            writer = csv.DictWriter(fh, fieldnames=CSV_FIELDS)
            writer.writeheader()
            writer.writerow(row)
        self.log(f"  Metrics: {path}")
