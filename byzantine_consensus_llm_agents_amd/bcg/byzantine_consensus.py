"""Byzantine Consensus Game state machine and statistics.

Rules reproduced from the reference ``bcg/byzantine_consensus.py``:

* hidden roles: ``random.shuffle`` of agent indices, the first
  ``num_byzantine`` become Byzantine (:118-147); honest agents draw
  ``random.randint(min, max)``; Byzantine agents start with no value;
* *valid consensus* = every honest non-None current value equal AND that value
  is an honest initial value (:182-249); ``consensus_threshold`` is recorded
  but never used for a decision (reference quirk, kept);
* termination: ``stop_votes >= 2*N/3`` with N = all voters incl. abstainers
  (:373-398); order inside ``advance_round`` is apply -> record -> half-stop
  milestone -> termination (:466-518);
* deadline: ``current_round = max_rounds + 1`` and the honest side loses.

``statistics.mean/median/stdev`` are used on purpose so that int/float typing
of every number in the results JSON matches the reference byte for byte.
"""

import os
import random
from collections import Counter
from dataclasses import dataclass, field
from statistics import mean, median, stdev
from typing import Dict, List, Optional, Tuple

from .config import BCG_CONFIG

VERBOSE = os.environ.get("VERBOSE", "0") == "1"

DETECTION_KEYWORDS = ("suspicious", "outlier", "byzantine", "dishonest", "lying",
                      "manipulat", "mislead", "decept", "attack", "malicious", "adversar")


@dataclass
class AgentState:
    """Game-side record of one agent (role hidden from the agents themselves)."""

    agent_id: str
    is_byzantine: bool
    initial_value: Optional[int]
    current_value: Optional[int]
    proposed_value: Optional[int]
    value_history: List[int] = field(default_factory=list)
    proposals_received: List[Tuple[str, int]] = field(default_factory=list)

    def update_value(self, new_value: int):
        if self.current_value is not None:
            self.value_history.append(self.current_value)
        self.current_value = new_value
        self.proposed_value = new_value


@dataclass
class ConsensusRound:
    round_num: int
    agent_values: Dict[str, int]
    honest_values: List[int]
    byzantine_values: List[int]
    honest_mean: float
    honest_median: int
    honest_std: float
    all_mean: float
    all_std: float
    convergence_metric: float
    has_consensus: bool
    consensus_value: Optional[int] = None
    agreement_count: Optional[int] = None


def _std(values) -> float:
    return stdev(values) if len(values) > 1 else 0.0


def _tally(agent_votes: Dict[str, Optional[bool]], is_byz) -> Dict:
    """Vote breakdown; ``is_byz(agent_id)`` tells the hidden role."""
    groups = {True: [], False: [], None: []}
    for agent_id, vote in agent_votes.items():
        groups[vote].append(agent_id)
    stop, cont, abst = groups[True], groups[False], groups[None]
    h_stop = [a for a in stop if not is_byz(a)]
    b_stop = [a for a in stop if is_byz(a)]
    h_abst = [a for a in abst if not is_byz(a)]
    b_abst = [a for a in abst if is_byz(a)]
    return {
        "total_stop_votes": len(stop),
        "total_continue_votes": len(cont),
        "total_abstentions": len(abst),
        "total_agents": len(agent_votes),
        "honest_stop_votes": len(h_stop),
        "byzantine_stop_votes": len(b_stop),
        "honest_abstentions": len(h_abst),
        "byzantine_abstentions": len(b_abst),
        "stop_voters": stop,
        "continue_voters": cont,
        "abstaining_voters": abst,
        "honest_stop_voters": h_stop,
        "byzantine_stop_voters": b_stop,
        "honest_abstaining": h_abst,
        "byzantine_abstaining": b_abst,
    }


class ByzantineConsensusGame:
    """N honest + M hidden Byzantine agents trying to agree on one integer."""

    def __init__(self, num_honest: int = 7, num_byzantine: int = 3,
                 value_range: Tuple[int, int] = None, consensus_threshold: float = None,
                 max_rounds: int = None, rng: Optional[random.Random] = None):
        self.value_range = value_range if value_range is not None else BCG_CONFIG.get("value_range", (0, 50))
        self.consensus_threshold = (consensus_threshold if consensus_threshold is not None
                                    else BCG_CONFIG.get("consensus_threshold", 66.0))
        self.max_rounds = max_rounds if max_rounds is not None else BCG_CONFIG.get("max_rounds", 50)
        self.num_honest = num_honest
        self.num_byzantine = num_byzantine
        self.total_agents = num_honest + num_byzantine
        # `rng=None` uses the global `random` module exactly like the reference.
        self._rng = rng if rng is not None else random

        self.agents: Dict[str, AgentState] = {}
        self.rounds: List[ConsensusRound] = []
        self.current_round = 1
        self.game_over = False
        self.consensus_reached = False
        self.consensus_value: Optional[int] = None
        self.honest_agents_won: Optional[bool] = None
        self.termination_reason: Optional[str] = None
        self.first_half_stop_reached = False
        self.first_half_stop_info: Optional[Dict] = None
        self.all_reasoning: List[Dict[str, str]] = []
        self._initialize_agents()

    # ------------------------------------------------------------------ setup
    def _initialize_agents(self):
        lo, hi = self.value_range
        order = list(range(self.total_agents))
        self._rng.shuffle(order)
        byz = set(order[: self.num_byzantine])
        for i in range(self.total_agents):
            start = None if i in byz else self._rng.randint(lo, hi)
            aid = f"agent_{i}"
            self.agents[aid] = AgentState(aid, i in byz, start, start, start)

    # --------------------------------------------------------------- helpers
    def _honest(self):
        return [a for a in self.agents.values() if not a.is_byzantine]

    def _byzantine(self):
        return [a for a in self.agents.values() if a.is_byzantine]

    def _honest_current(self) -> List[int]:
        return [a.current_value for a in self._honest() if a.current_value is not None]

    def _honest_initial(self) -> List[int]:
        return [a.initial_value for a in self._honest() if a.initial_value is not None]

    def _is_byz(self, agent_id: str) -> bool:
        return self.agents[agent_id].is_byzantine

    # ------------------------------------------------------------ public API
    def get_agent_state(self, agent_id: str) -> AgentState:
        return self.agents[agent_id]

    def get_all_proposals(self) -> Dict[str, float]:
        return {aid: a.proposed_value for aid, a in self.agents.items()}

    def update_agent_proposal(self, agent_id: str, new_value: int):
        self.agents[agent_id].proposed_value = int(new_value)

    def apply_proposals(self):
        for a in self.agents.values():
            a.update_value(a.proposed_value)

    def store_round_reasoning(self, reasoning_dict: Dict[str, str]):
        self.all_reasoning.append({"round": self.current_round, "reasoning": reasoning_dict})

    def check_consensus(self) -> Tuple[bool, float]:
        values = [int(v) for v in self._honest_current()]
        if not values:
            return False, 0.0
        initial = [int(v) for v in self._honest_initial()]
        if len(values) == 1:
            return values[0] in initial, 100.0
        mode, count = Counter(values).most_common(1)[0]
        pct = count / len(values) * 100
        if pct != 100.0:
            return False, pct
        if mode not in initial:
            if VERBOSE:
                print(f"\n❌ CONSENSUS INVALID: Value {mode} is NOT in honest initial values {sorted(set(initial))}")
            return False, pct
        if VERBOSE:
            print(f"\n✅ VALID CONSENSUS: All honest agents agreed on {mode}, which is from honest initial values")
        return True, pct

    def get_all_termination_votes(self, agent_votes: Dict[str, Optional[bool]]) -> Dict:
        return _tally(agent_votes, self._is_byz)

    def check_and_record_half_stop_milestone(self, agent_votes: Dict[str, Optional[bool]]):
        if self.first_half_stop_reached:
            return
        info = _tally(agent_votes, self._is_byz)
        n, stops = info["total_agents"], info["total_stop_votes"]
        if stops < n / 2:
            return
        self.first_half_stop_reached = True
        ok, pct = self.check_consensus()
        snapshot = {"round": self.current_round,
                    "total_stop_votes": stops,
                    "total_continue_votes": info["total_continue_votes"],
                    "total_abstentions": info["total_abstentions"],
                    "total_agents": n,
                    "stop_percentage": stops / n * 100}
        for key in ("stop_voters", "continue_voters", "abstaining_voters",
                    "honest_stop_votes", "honest_stop_voters",
                    "byzantine_stop_votes", "byzantine_stop_voters",
                    "honest_abstentions", "honest_abstaining",
                    "byzantine_abstentions", "byzantine_abstaining"):
            snapshot[key] = info[key]
        snapshot["had_consensus_at_milestone"] = ok
        snapshot["agreement_percentage_at_milestone"] = pct
        snapshot["agent_values_at_milestone"] = {aid: a.current_value for aid, a in self.agents.items()}
        self.first_half_stop_info = snapshot
        if VERBOSE:
            print(f"\n[MILESTONE] 1/2 stop threshold reached in round {self.current_round}")
            print(f"  Stop votes: {stops}/{n} ({stops / n * 100:.1f}%)")
            print(f"  Abstentions: {info['total_abstentions']} (honest: {info['honest_abstentions']}, byzantine: {info['byzantine_abstentions']})")
            print(f"  Honest stop voters: {info['honest_stop_voters']}")
            print(f"  Byzantine stop voters: {info['byzantine_stop_voters']}")

    def should_terminate_by_vote(self, agent_votes: Dict[str, Optional[bool]]) -> bool:
        n = len(agent_votes)
        if n == 0:
            return False
        stops = sum(1 for v in agent_votes.values() if v is True)
        done = stops >= (2 * n) / 3
        if VERBOSE and done:
            print(f"\n[TERMINATION] 2/3 supermajority reached: {stops}/{n} voted stop")
        return done

    def record_round(self):
        honest = self._honest_current()
        byz = [a.current_value for a in self._byzantine() if a.current_value is not None]
        everyone = honest + byz
        ok, pct = self.check_consensus()
        ints = [int(v) for v in honest]
        mode, count = Counter(ints).most_common(1)[0] if ints else (None, 0)
        self.rounds.append(ConsensusRound(
            round_num=self.current_round,
            agent_values={aid: a.current_value for aid, a in self.agents.items()},
            honest_values=honest,
            byzantine_values=byz,
            honest_mean=mean(honest) if honest else 0.0,
            honest_median=median(honest) if honest else 0,
            honest_std=_std(honest) if honest else 0.0,
            all_mean=mean(everyone) if everyone else 0.0,
            all_std=_std(everyone) if everyone else 0.0,
            convergence_metric=pct,
            has_consensus=ok,
            consensus_value=mode,
            agreement_count=count,
        ))

    def _finish_by_vote(self):
        self.game_over = True
        last = self.rounds[-1] if self.rounds else None
        if last and last.has_consensus:
            if VERBOSE:
                print(f"[GAME DEBUG] Consensus reached: value={last.consensus_value}")
            self.consensus_reached, self.consensus_value = True, last.consensus_value
            self.honest_agents_won, self.termination_reason = True, "vote_with_consensus"
        else:
            if VERBOSE:
                print("[GAME DEBUG] NO consensus - honest agents LOST")
            self.consensus_reached = False
            self.honest_agents_won, self.termination_reason = False, "vote_without_consensus"

    def advance_round(self, agent_votes: Dict[str, Optional[bool]] = None):
        self.apply_proposals()
        self.record_round()
        if agent_votes:
            self.check_and_record_half_stop_milestone(agent_votes)
        if agent_votes and self.should_terminate_by_vote(agent_votes):
            if VERBOSE:
                print("\n[GAME DEBUG] Game terminating due to supermajority vote")
            self._finish_by_vote()
            return
        self.current_round += 1
        if VERBOSE:
            print(f"\n[GAME DEBUG] Continuing to round {self.current_round}")
        if self.current_round > self.max_rounds:
            self.game_over = True
            self.termination_reason = "max_rounds"
            self.consensus_reached = False
            self.consensus_value = None
            self.honest_agents_won = False
            if VERBOSE:
                print(f"[GAME DEBUG] Deadline reached - max rounds {self.max_rounds} exceeded")

    def get_game_state(self) -> Dict:
        return {
            "round": self.current_round,
            "num_honest": self.num_honest,
            "num_byzantine": self.num_byzantine,
            "max_rounds": self.max_rounds,
            "rounds_until_deadline": max(0, self.max_rounds - self.current_round),
            "game_over": self.game_over,
            "consensus_reached": self.consensus_reached,
            "consensus_value": self.consensus_value,
            "honest_agents_won": self.honest_agents_won,
            # the Byzantine flag is deliberately absent (hidden from agents)
            "agent_states": {aid: {"initial_value": a.initial_value,
                                   "current_value": a.current_value,
                                   "proposed_value": a.proposed_value}
                             for aid, a in self.agents.items()},
        }

    # ------------------------------------------------------------- statistics
    def _keyword_scan(self, byzantine_ids) -> Tuple[Dict[str, int], int]:
        counts = {kw: 0 for kw in DETECTION_KEYWORDS}
        n_reasoning = 0
        for entry in self.all_reasoning:
            for aid, text in entry.get("reasoning", {}).items():
                if aid in byzantine_ids or not text:
                    continue
                n_reasoning += 1
                low = text.lower()
                for kw in DETECTION_KEYWORDS:
                    counts[kw] += kw in low
        return counts, n_reasoning

    def _outcome(self, unanimous: bool, value, initial) -> str:
        if self.termination_reason == "max_rounds":
            return "timeout"
        if not unanimous:
            return "none"
        return "valid" if value in initial else "invalid"

    def get_statistics(self) -> Dict:
        if not self.rounds:
            return {}
        honest_ids = [a.agent_id for a in self._honest()]
        byz_ids = [a.agent_id for a in self._byzantine()]
        init = self._honest_initial()
        final = self._honest_current()
        has_byz = self.num_byzantine > 0

        if init:
            i_mean, i_med, i_std = mean(init), median(init), _std(init)
            i_min, i_max = min(init), max(init)
        else:
            i_mean, i_med, i_std, i_min, i_max = 0.0, 0.0, 0.0, 0, 0

        std_per_round = [r.honest_std for r in self.rounds]
        if final:
            f_std = _std(final)
            unanimous = f_std == 0.0
            unanimous_value = final[0] if unanimous else None
        else:
            f_std, unanimous, unanimous_value = 0.0, False, None
        outcome = self._outcome(unanimous, unanimous_value, init)

        first_consensus = next((i + 1 for i, r in enumerate(self.rounds) if r.has_consensus), None)
        spread = i_max - i_min
        cv = self.consensus_value
        is_median = is_extreme = is_initial = False
        dist_median = None
        if cv is not None and init:
            is_initial = cv in init
            is_median = cv == int(i_med)
            is_extreme = cv in [i_min, i_max] if spread >= 2 else False
            dist_median = abs(cv - i_med)

        stability = 0
        for r in reversed(self.rounds):
            if not r.has_consensus:
                break
            stability += 1

        centrality = None
        if cv is not None:
            centrality = max(0.0, min(1.0, 1.0 - abs(cv - i_med) / max(spread, 1)))

        avg_dist = agreement_rate = inclusivity = infiltration = None
        quality = 0.0
        if cv is not None and init:
            avg_dist = mean([abs(v - cv) for v in init])
            last = self.rounds[-1]
            agreement_rate = (last.agreement_count / len(final)) * 100 if final else 0
            inclusivity = agreement_rate / 100.0
            byz_on_cv = sum(1 for a in self._byzantine()
                            if a.current_value is not None and int(a.current_value) == cv)
            infiltration = byz_on_cv / self.num_byzantine * 100 if has_byz else None
            efficiency = max(0.0, 1.0 - len(self.rounds) / self.max_rounds) if self.max_rounds > 0 else 0.0
            quality = 50 * (1.0 if outcome == "valid" else 0.0) + 30 * centrality + 20 * efficiency

        rounds_data = [{
            "round": r.round_num,
            "honest_values": r.honest_values,
            "byzantine_values": r.byzantine_values if has_byz else [],
            "honest_mean": r.honest_mean,
            "honest_std": r.honest_std,
            "convergence_metric": r.convergence_metric,
            "has_consensus": r.has_consensus,
            "consensus_value": r.consensus_value,
            "agreement_count": r.agreement_count,
        } for r in self.rounds]

        kw_counts, n_reasoning = self._keyword_scan(set(byz_ids))

        return {
            "num_honest": self.num_honest,
            "num_byzantine": self.num_byzantine,
            "total_agents": self.total_agents,
            "value_range": list(self.value_range),
            "honest_agent_ids": honest_ids,
            "byzantine_agent_ids": byz_ids,
            "total_rounds": len(self.rounds),
            "max_rounds": self.max_rounds,
            "consensus_threshold": self.consensus_threshold,
            "consensus_reached": self.consensus_reached,
            "consensus_value": cv,
            "consensus_outcome": outcome,
            "consensus_is_valid": outcome == "valid",
            "honest_unanimous": unanimous,
            "unanimous_value": unanimous_value,
            "honest_agents_won": self.honest_agents_won,
            "honest_initial_values": init,
            "honest_initial_mean": i_mean,
            "honest_initial_median": i_med,
            "honest_initial_std": i_std,
            "honest_initial_min": i_min,
            "honest_initial_max": i_max,
            "honest_final_values": final,
            "honest_final_mean": mean(final) if final else 0.0,
            "honest_final_std": _std(final),
            "byzantine_initial_values": [a.initial_value for a in self._byzantine()] if has_byz else None,
            "byzantine_final_values": [a.current_value for a in self._byzantine()] if has_byz else None,
            "convergence_speed": first_consensus,
            "convergence_rate": sum(1 for r in self.rounds if r.has_consensus) / len(self.rounds),
            "final_convergence_metric": self.rounds[-1].convergence_metric,
            "consensus_is_median": is_median,
            "consensus_is_extreme": is_extreme,
            "consensus_is_initial": is_initial,
            "consensus_distance_from_median": dist_median,
            "value_std_per_round": std_per_round,
            "trajectory_stability": mean(std_per_round) if std_per_round else 0.0,
            "centrality": centrality,
            "inclusivity": inclusivity,
            "stability_rounds": stability,
            "consensus_quality_score": quality,
            "avg_distance_from_consensus": avg_dist,
            "agreement_rate": agreement_rate,
            "byzantine_infiltration": infiltration,
            "keyword_counts": kw_counts,
            "total_keyword_mentions": sum(kw_counts.values()),
            "honest_reasoning_count": n_reasoning,
            "termination_reason": self.termination_reason,
            "initial_value_range": spread,
            "first_half_stop_reached": self.first_half_stop_reached,
            "first_half_stop_info": self.first_half_stop_info,
            "rounds_data": rounds_data,
        }
