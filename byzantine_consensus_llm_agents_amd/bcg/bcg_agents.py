"""LLM agents of the Byzantine Consensus Game.

Behavioural parity with reference ``bcg/bcg_agents.py``:

* agent-side memory (``AgentState`` :86-131): rolling round summaries and up to
  5 internal-strategy notes (trimmed to 400 chars); only the last 3 summaries
  are rendered, newest first (:271-285);
* honest / Byzantine prompt + schema builders used by the batched simulator
  path, and the parsers applied to batched results (:577-681, :1069-1191);
* the sequential 3-attempt paths with ``RETRY ATTEMPT k/3`` suffixes used by
  the simulator's per-agent retry (:683-876, :1193-1399);
* module-level tee logging (``set_agent_log_file`` / ``print`` / ``verbose_print``).

Role differences are expressed as a small table of hooks on each subclass
instead of duplicated methods.
"""

import builtins
import json
from collections import defaultdict
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

from . import prompts as P
from .config import LLM_CONFIG
from .engine_agent import VERBOSE, EngineAgent

_agent_log_file = None
_builtin_print = builtins.print

MAX_HISTORY_ROUNDS = 5
MAX_JSON_RETRIES = 3  # hard-coded in the reference (LLM_CONFIG['max_json_retries'] is ignored)


def set_agent_log_file(file_handle):
    global _agent_log_file
    _agent_log_file = file_handle


def print(*args, **kwargs):  # noqa: A001 - module-level tee, as in the reference
    _builtin_print(*args, **kwargs)
    if _agent_log_file:
        _builtin_print(*args, **kwargs, file=_agent_log_file, flush=True)


def verbose_print(*args, **kwargs):
    if _agent_log_file:
        _builtin_print(*args, **kwargs, file=_agent_log_file, flush=True)
    if VERBOSE:
        _builtin_print(*args, **kwargs)


@dataclass
class AgentState:
    """Agent-side persistent memory across rounds."""

    last_k_rounds: List[str] = field(default_factory=list)
    last_k_internal_strategies: List[Tuple[int, str]] = field(default_factory=list)
    neighbor_stats: Dict[str, dict] = field(default_factory=lambda: defaultdict(dict))
    current_goal: str = "REACH_CONSENSUS"
    local_state: Dict = field(default_factory=dict)

    @staticmethod
    def _push(buf: list, item, cap: int):
        buf.append(item)
        if len(buf) > cap:
            buf.pop(0)

    def add_round_summary(self, summary: str, max_history: int = MAX_HISTORY_ROUNDS):
        self._push(self.last_k_rounds, summary, max_history)

    def add_internal_strategy(self, round_num: int, strategy: str, max_history: int = MAX_HISTORY_ROUNDS):
        self._push(self.last_k_internal_strategies, (round_num, strategy), max_history)

    def update_neighbor_stat(self, agent_id: str, value: int):
        st = self.neighbor_stats.get(agent_id)
        if st is None or agent_id not in self.neighbor_stats:
            self.neighbor_stats[agent_id] = {"last_value": value, "message_count": 0}
        else:
            st["last_value"] = value
            st["message_count"] = st.get("message_count", 0) + 1


class BCGAgent(EngineAgent):
    """Shared machinery; subclasses provide the role hooks."""

    # role hooks (overridden by subclasses)
    vote_options: Tuple[str, ...] = P.HONEST_VOTE_OPTIONS
    decide_retry_template: str = P.RETRY_HONEST_DECIDE
    log_tag: str = ""

    def __init__(self, agent_id: str, is_byzantine: bool, model_name: str = "Qwen/Qwen3-14B",
                 model_config: Optional[Dict] = None, value_range: Optional[tuple] = None,
                 byzantine_awareness: str = "may_exist"):
        super().__init__(agent_id, model_name, model_config)
        self.is_byzantine = is_byzantine
        self.value_range = value_range
        self.byzantine_awareness = byzantine_awareness
        self.initial_value = None
        self.my_value = None
        self.received_proposals: List[Tuple[str, int, str]] = []
        self.last_reasoning = ""
        self.a2a_client = None
        self.state = AgentState()
        self.state.current_goal = "DISRUPT_CONSENSUS" if is_byzantine else "REACH_CONSENSUS"
        self._cached_system_prompt: Optional[str] = None
        self._cached_vote_system_prompt: Optional[str] = None

    # ---------------------------------------------------------------- state
    def set_a2a_client(self, client):
        self.a2a_client = client

    def set_initial_value(self, value: int):
        self.initial_value = value
        self.my_value = value
        self._cached_system_prompt = None
        self._cached_vote_system_prompt = None

    def receive_proposals(self, proposals: List[Tuple[str, int, str]]):
        self.received_proposals = proposals
        for sender, value, _ in proposals:
            self.state.update_neighbor_stat(sender, value)

    def _record_internal_strategy(self, round_num: int, strategy: str):
        trimmed = strategy.strip()[:400] if strategy else ""
        if trimmed:
            self.state.add_internal_strategy(round_num, trimmed)

    def _format_strategy_history(self, history: Optional[List[Tuple[int, str]]] = None) -> str:
        entries = self.state.last_k_internal_strategies if history is None else history
        return "\n".join(f"round {r}: {note}" for r, note in entries)

    def _format_history_with_agent_details(self, max_rounds: int = 3) -> str:
        rounds = self.state.last_k_rounds
        if not rounds:
            return P.NO_HISTORY
        return "\n".join(reversed(rounds[-max_rounds:]))

    def _notes(self, empty: str) -> str:
        notes = self._format_strategy_history() if self.state.last_k_internal_strategies else ""
        return notes if notes else empty

    def _range(self):
        lo, hi = self.value_range
        return lo, hi

    def _clamp(self, value) -> int:
        lo, hi = self._range()
        return int(max(lo, min(hi, value)))

    # --------------------------------------------------------- prompt hooks
    def build_system_prompt(self, game_state: Dict) -> str:
        raise NotImplementedError

    def build_round_prompt(self, game_state: Dict) -> str:
        raise NotImplementedError

    def build_vote_system_prompt(self, game_state: Dict) -> str:
        raise NotImplementedError

    def build_vote_round_prompt(self, game_state: Dict) -> str:
        raise NotImplementedError

    def decision_schema(self) -> Dict:
        raise NotImplementedError

    def vote_schema(self) -> Dict:
        return P.vote_schema(self.vote_options)

    def _decision_ok(self, result: Dict) -> bool:
        raise NotImplementedError

    def _apply_decision(self, result: Dict, round_num: int, default_reasoning: str) -> Optional[int]:
        raise NotImplementedError

    # ------------------------------------------------------ batched helpers
    def build_decision_prompt(self, game_state: Dict) -> Optional[Tuple[str, str, Dict]]:
        return (self.build_system_prompt(game_state), self.build_round_prompt(game_state),
                self.decision_schema())

    def build_vote_prompt(self, game_state: Dict) -> Tuple[str, str, Dict]:
        return (self.build_vote_system_prompt(game_state), self.build_vote_round_prompt(game_state),
                self.vote_schema())

    def parse_decision_response(self, result: Dict, game_state: Dict) -> Optional[int]:
        if result is None or "error" in result:
            verbose_print(f"❌ [{self.agent_id}] {self.log_tag}JSON PARSING FAILED - NO PARTICIPATION THIS ROUND")
            self.last_reasoning = "⚠️ JSON PARSING FAILED - no response"
            return None
        return self._apply_decision(result, game_state.get("round", 0), self._batched_default_reasoning)

    def _vote_value(self, decision: str) -> Optional[bool]:
        if decision == "stop":
            return True
        if decision == "abstain" and "abstain" in self.vote_options:
            return None
        return False

    def parse_vote_response(self, result: Dict, game_state: Dict) -> Optional[bool]:
        if result is None or "error" in result:
            verbose_print(f"❌ [{self.agent_id}] {self.log_tag}VOTE JSON FAILED - DEFAULTING TO CONTINUE")
            return False
        vote = self._vote_value(result.get("decision", "continue").lower().strip())
        verbose_print(f"🗳️  [{self.agent_id} VOTE] -> {'STOP' if vote else ('ABSTAIN' if vote is None else 'CONTINUE')}")
        return vote

    # ---------------------------------------------------- sequential paths
    def step(self, round_t: int, phase: str, game_state: Dict) -> Optional[int]:
        return self.decide_next_value(game_state)

    def _ask_with_retries(self, system_prompt: str, base_prompt: str, schema: Dict,
                          temperature: float, max_tokens: int, accept, retry_text) -> Optional[Dict]:
        """Up to 3 attempts; the prompt gets a RETRY suffix after a failure."""
        prompt = base_prompt
        result = None
        for attempt in range(1, MAX_JSON_RETRIES + 1):
            self.sequential_attempts = getattr(self, "sequential_attempts", 0) + 1  # (retry cost counter)
            result = self.generate_json(prompt, schema, temperature=temperature,
                                        max_tokens=max_tokens, system_prompt=system_prompt)
            verbose_print(f"🔍 [{self.agent_id} attempt {attempt}] {json.dumps(result)}")
            if "error" not in result:
                if accept(result):
                    return result
                result = {"error": "invalid_fields"}
            if attempt < MAX_JSON_RETRIES:
                prompt = retry_text(base_prompt, attempt + 1)
        return None

    def decide_next_value(self, game_state: Dict) -> Optional[int]:
        result = self._ask_with_retries(
            self.build_system_prompt(game_state), self.build_round_prompt(game_state),
            self.decision_schema(), LLM_CONFIG["temperature_decide"], LLM_CONFIG["max_tokens_decide"],
            self._decision_ok,
            lambda base, nxt: self.decide_retry_template.format(base=base, next=nxt, total=MAX_JSON_RETRIES))
        if result is None:
            self._on_decide_exhausted()
            self.last_reasoning = f"⚠️ JSON PARSING FAILED ({MAX_JSON_RETRIES} attempts) - no response"
            return None
        return self._apply_decision(result, game_state.get("round", 0), self._sequential_default_reasoning)

    def _on_decide_exhausted(self):
        verbose_print(f"❌ [{self.agent_id}] FAILED ALL {MAX_JSON_RETRIES} JSON ATTEMPTS - NO PARTICIPATION THIS ROUND")

    def vote_to_terminate(self, game_state: Dict) -> Optional[bool]:
        options = self.vote_options

        def accept(res):
            d = res.get("decision", "")
            return bool(d) and d.strip() in options

        result = self._ask_with_retries(
            self.build_vote_system_prompt(game_state), self.build_vote_round_prompt(game_state),
            self.vote_schema(), LLM_CONFIG["temperature_vote"], LLM_CONFIG["max_tokens_vote"], accept,
            lambda base, nxt: P.RETRY_VOTE.format(base=base, next=nxt, total=MAX_JSON_RETRIES,
                                                  options=P.quoted_options(options)))
        # whether the vote came from a valid response (False: all attempts failed and the
        # reference's default CONTINUE is returned) -- read by the decisions/s counter only
        self.last_vote_valid = result is not None
        if result is None:
            verbose_print(f"❌ [{self.agent_id}] FAILED ALL {MAX_JSON_RETRIES} JSON ATTEMPTS - DEFAULTING TO CONTINUE")
            return False
        return self._vote_value(result.get("decision", "continue").lower().strip())


class HonestBCGAgent(BCGAgent):
    """Honest agent: converge on one of the honest initial values."""

    vote_options = P.HONEST_VOTE_OPTIONS
    decide_retry_template = P.RETRY_HONEST_DECIDE
    _batched_default_reasoning = "Value proposed"
    _sequential_default_reasoning = "Value proposed"

    def _cooperative(self) -> bool:
        return self.byzantine_awareness == "none_exist"

    def build_system_prompt(self, game_state: Dict) -> str:
        if self._cached_system_prompt is None:
            lo, hi = self._range()
            tpl = P.HONEST_SYSTEM_COOPERATIVE if self._cooperative() else P.HONEST_SYSTEM_BYZANTINE_AWARE
            self._cached_system_prompt = tpl.format(
                agent_id=self.agent_id, max_rounds=game_state.get("max_rounds", 20),
                lo=lo, hi=hi, initial=int(self.initial_value))
        return self._cached_system_prompt

    def build_round_prompt(self, game_state: Dict) -> str:
        return P.HONEST_ROUND.format(
            round=game_state.get("round", 0), state_line=P.state_line(self.my_value),
            history=self._format_history_with_agent_details(3), notes=self._notes("(No notes yet)"))

    def build_vote_system_prompt(self, game_state: Dict) -> str:
        if self._cached_vote_system_prompt is None:
            tpl = P.HONEST_VOTE_SYSTEM_COOPERATIVE if self._cooperative() else P.HONEST_VOTE_SYSTEM_BYZANTINE_AWARE
            self._cached_vote_system_prompt = tpl.format(
                agent_id=self.agent_id, max_rounds=game_state.get("max_rounds", 20))
        return self._cached_vote_system_prompt

    def build_vote_round_prompt(self, game_state: Dict) -> str:
        return P.HONEST_VOTE_ROUND.format(
            round=game_state.get("round", 0), max_rounds=game_state.get("max_rounds", 20),
            proposals=P.proposals_block(self.agent_id, self.my_value, self.last_reasoning,
                                        self.received_proposals),
            history=P.vote_history(self._format_history_with_agent_details(3)),
            notes=self._notes("(No notes)"))

    def decision_schema(self) -> Dict:
        return P.honest_decision_schema(*self._range())

    def _decision_ok(self, result: Dict) -> bool:
        return (result.get("value") is not None
                and len(result.get("internal_strategy", "").strip()) > 0
                and len(result.get("public_reasoning", "").strip()) > 0)

    def _apply_decision(self, result: Dict, round_num: int, default_reasoning: str) -> Optional[int]:
        value = result.get("value")
        if value is None:
            self.last_reasoning = "⚠️ No value provided - agent abstains"
            return None
        self.last_reasoning = result.get("public_reasoning", default_reasoning)[:600]
        self._record_internal_strategy(round_num, result.get("internal_strategy", ""))
        return self._clamp(value)

    def _on_decide_exhausted(self):
        # the honest path reports this on the console (print), Byzantine only logs it
        print(f"❌ [{self.agent_id}] FAILED ALL {MAX_JSON_RETRIES} JSON ATTEMPTS - NO PARTICIPATION THIS ROUND")


class ByzantineBCGAgent(BCGAgent):
    """Hidden adversary: may abstain on value and vote."""

    vote_options = P.BYZANTINE_VOTE_OPTIONS
    decide_retry_template = P.RETRY_BYZANTINE_DECIDE
    log_tag = "BYZANTINE "
    _batched_default_reasoning = "Adjusting my position."
    _sequential_default_reasoning = "Adjusting my position."

    def __init__(self, agent_id: str, is_byzantine: bool = True, model_name: str = "Qwen/Qwen-3-14B",
                 model_config: Optional[Dict] = None, value_range: Optional[tuple] = None,
                 byzantine_awareness: str = "may_exist"):
        super().__init__(agent_id, is_byzantine, model_name, model_config, value_range, byzantine_awareness)

    def build_system_prompt(self, game_state: Dict) -> str:
        if self._cached_system_prompt is None:
            lo, hi = self._range()
            self._cached_system_prompt = P.BYZANTINE_SYSTEM.format(
                agent_id=self.agent_id, max_rounds=game_state.get("max_rounds", 20), lo=lo, hi=hi)
        return self._cached_system_prompt

    def build_round_prompt(self, game_state: Dict) -> str:
        return P.BYZANTINE_ROUND.format(
            round=game_state.get("round", 0), state_line=P.state_line(self.my_value),
            history=self._format_history_with_agent_details(3), notes=self._notes("(No notes yet)"))

    def build_vote_system_prompt(self, game_state: Dict) -> str:
        if self._cached_vote_system_prompt is None:
            self._cached_vote_system_prompt = P.BYZANTINE_VOTE_SYSTEM.format(
                agent_id=self.agent_id, max_rounds=game_state.get("max_rounds", 20))
        return self._cached_vote_system_prompt

    def build_vote_round_prompt(self, game_state: Dict) -> str:
        return P.BYZANTINE_VOTE_ROUND.format(
            round=game_state.get("round", 0), max_rounds=game_state.get("max_rounds", 20),
            proposals=P.proposals_block(self.agent_id, self.my_value, self.last_reasoning,
                                        self.received_proposals),
            history=P.vote_history(self._format_history_with_agent_details(3)))

    def decision_schema(self) -> Dict:
        return P.byzantine_decision_schema(*self._range())

    def _decision_ok(self, result: Dict) -> bool:
        value = result.get("value")
        return (len(result.get("internal_strategy", "").strip()) > 0
                and (isinstance(value, int) or value == "abstain"))

    def _apply_decision(self, result: Dict, round_num: int, default_reasoning: str) -> Optional[int]:
        strategy = result.get("internal_strategy", "")
        if strategy:
            self._record_internal_strategy(round_num, strategy)
        value = result.get("value")
        reasoning = result.get("public_reasoning")
        if value == "abstain" or value is None:
            verbose_print(f"🔇 [{self.agent_id}] BYZANTINE CHOSE TO ABSTAIN this round")
            self.last_reasoning = reasoning[:600] if reasoning else ""
            return None
        if not isinstance(value, int):
            self.last_reasoning = ""
            return None
        self.last_reasoning = result.get("public_reasoning", default_reasoning)[:600]
        return self._clamp(value)


def create_agent(agent_id: str, is_byzantine: bool,
                 model_name: str = "meta-llama/Meta-Llama-3.1-8B-Instruct",
                 model_config: Optional[Dict] = None, value_range: Optional[tuple] = None,
                 byzantine_awareness: str = "may_exist") -> BCGAgent:
    cls = ByzantineBCGAgent if is_byzantine else HonestBCGAgent
    return cls(agent_id, is_byzantine, model_name, model_config, value_range, byzantine_awareness)
