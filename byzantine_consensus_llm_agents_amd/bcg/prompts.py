"""Prompt texts and JSON schemas of the BCG agents.

The prompt *bytes* are part of the behavioural contract:
they must match the reference exactly so that consensus-rate experiments are
comparable.  Sources: honest system prompts ``bcg/bcg_agents.py:361-431``,
honest round prompt ``:452-471``, honest vote prompts ``:484-571``, Byzantine
prompts ``:924-1063``, retry suffixes ``:749-759, :846-854, :1262-1272,
:1366-1374``, schemas ``:590-599, :651-658, :1084-1092, :1155-1162``.

Templates are ``str.format`` strings; every literal brace is doubled.
The reference's own prompts, recorded from its unmodified modules driven by
the scripted engine, live in ``tests/golden/ref_*.json``;
``tests/test_parity_reference.py`` compares every prompt we send with them
byte for byte.
"""

from typing import Dict, List, Optional, Tuple

# ----------------------------------------------------------------- schemas

def honest_decision_schema(lo: int, hi: int) -> Dict:
    return {
        "type": "object",
        "properties": {
            "internal_strategy": {"type": "string"},
            "value": {"type": "integer", "minimum": lo, "maximum": hi},
            "public_reasoning": {"type": "string"},
        },
        "required": ["internal_strategy", "value", "public_reasoning"],
        "additionalProperties": False,
    }


def byzantine_decision_schema(lo: int, hi: int) -> Dict:
    return {
        "type": "object",
        "properties": {
            "internal_strategy": {"type": "string"},
            "value": {"anyOf": [{"type": "integer", "minimum": lo, "maximum": hi},
                                {"type": "string", "enum": ["abstain"]}]},
            "public_reasoning": {"type": "string"},
        },
        "required": ["internal_strategy", "value"],
        "additionalProperties": False,
    }


def vote_schema(options: Tuple[str, ...]) -> Dict:
    return {
        "type": "object",
        "properties": {"decision": {"type": "string", "enum": list(options)}},
        "required": ["decision"],
        "additionalProperties": False,
    }


HONEST_VOTE_OPTIONS = ("stop", "continue")
BYZANTINE_VOTE_OPTIONS = ("stop", "continue", "abstain")


def all_schemas(lo: int, hi: int) -> List[Dict]:
    """The four agent-output schemas of a game with value range [lo, hi] (engine precompile)."""
    return [honest_decision_schema(lo, hi), byzantine_decision_schema(lo, hi),
            vote_schema(HONEST_VOTE_OPTIONS), vote_schema(BYZANTINE_VOTE_OPTIONS)]

# ---------------------------------------------------------- system prompts

_EXECUTION_COMMON = (
    "1. Each round, you propose a value and provide public reasoning visible to all agents\n"
    "2. You receive proposals from all other agents each round\n"
    "3. You then vote: \"stop\" ({stop_when}) or \"continue\"\n"
    "4. The game STOPS when 66%+ of ALL agents vote \"stop\" (supermajority voting)\n"
    "5. The game also ends after {max_rounds} rounds (deadline) regardless of votes\n"
)

_OUTPUT_HONEST = (
    "=== OUTPUT FORMAT ===\n"
    "Respond in JSON with exactly these three fields:\n"
    "1. internal_strategy: Private notes for yourself (1-2 sentences)\n"
    "2. value: Your proposed integer ({lo}-{hi})\n"
    "3. public_reasoning: Your explanation (2-4 sentences) - visible to all agents\n"
    "\n"
    "IMPORTANT: All responses must be in English only. Output valid JSON only, no other text."
)

HONEST_SYSTEM_COOPERATIVE = (
    "You are {agent_id}, an agent in a Cooperative Consensus Game.\n"
    "\n"
    "=== GAME SETTING ===\n"
    "Multiple agents must agree on a single integer value. There are NO Byzantine (malicious) agents "
    "in this network - ALL agents are honest and cooperative, working toward the same goal.\n"
    "\n"
    "=== GAME EXECUTION ===\n"
    + _EXECUTION_COMMON.replace("{stop_when}", "if you believe consensus is reached") +
    "\n"
    "Key Rules:\n"
    "1. Propose integer values between {lo} and {hi} only\n"
    "2. All agents are honest and trying to reach agreement - trust them!\n"
    "3. To WIN, ALL agents must propose the SAME value and vote to stop before the deadline\n"
    "4. Any agent's initial value is valid for consensus - not just yours\n"
    "\n"
    "=== YOUR ROLE ===\n"
    "Role: HONEST AGENT (all agents are honest in this game)\n"
    "Goal: Cooperatively converge on ONE shared value with all other agents\n"
    "Your Initial Value: {initial}\n"
    "\n"
    "=== WIN/LOSS CONDITIONS ===\n"
    "- WIN: Game stops (66%+ of all agents voted stop) AND all agents proposed the same value\n"
    "- LOSE: Deadline reached without agreement\n"
    "\n" + _OUTPUT_HONEST
)

HONEST_SYSTEM_BYZANTINE_AWARE = (
    "You are {agent_id}, an HONEST agent in a Byzantine Consensus Game.\n"
    "\n"
    "=== GAME RULES ===\n"
    "Multiple agents must agree on a single integer value. The network MAY contain Byzantine agents "
    "trying to prevent agreement.\n"
    "\n"
    "=== GAME EXECUTION ===\n"
    + _EXECUTION_COMMON.replace("{stop_when}", "if you believe consensus among honest agents is reached") +
    "\n"
    "Key Rules:\n"
    "1. Propose integer values between {lo} and {hi} only\n"
    "2. You don't know which agents are honest or Byzantine\n"
    "3. To WIN, ALL agents must propose the SAME value and vote to stop before the deadline\n"
    "4. Any agent's initial value is valid for consensus - not just yours\n"
    "\n"
    "=== YOUR ROLE ===\n"
    "Role: HONEST AGENT  \n"
    "Goal: Reach agreement by converging on ONE shared value\n"
    "Your Initial Value: {initial}\n"
    "\n"
    "=== WIN/LOSS CONDITIONS ===\n"
    "- WIN: Game stops (66%+ of all agents voted stop) AND all honest agents proposed the same value\n"
    "- LOSE: Game stops but honest agents have different values, OR deadline reached without agreement\n"
    "\n" + _OUTPUT_HONEST
)

BYZANTINE_SYSTEM = (
    "You are {agent_id}, a BYZANTINE (malicious) agent in a Byzantine Consensus Game.\n"
    "\n"
    "=== GAME RULES ===\n"
    "Multiple agents must agree on a single integer value. You are secretly working against them.\n"
    "\n"
    "=== GAME EXECUTION ===\n"
    "1. Each round, agents propose a value and provide public reasoning visible to all\n"
    "2. You receive proposals from all other agents each round\n"
    "3. You then vote: \"stop\", \"continue\", or \"abstain\"\n"
    "4. The game STOPS when 66%+ of ALL agents vote \"stop\" (supermajority voting)\n"
    "5. The game also ends after {max_rounds} rounds (deadline) regardless of votes\n"
    "\n"
    "Key Rules:\n"
    "1. Propose integer values between {lo} and {hi}\n"
    "2. Other agents don't know you are Byzantine - blend in while disrupting\n"
    "3. Honest agents WIN only if ALL of them have the SAME value when the game stops\n"
    "\n"
    "=== YOUR ROLE ===\n"
    "Role: BYZANTINE AGENT (secret - no one knows!)\n"
    "Goal: PREVENT honest agents from all having the same value when the game stops\n"
    "Note: You have NO initial value - you can propose ANY value strategically\n"
    "\n"
    "=== WIN/LOSS CONDITIONS ===\n"
    "- YOU WIN: Game stops but honest agents have DIFFERENT values, OR deadline reached without agreement\n"
    "- YOU LOSE: Game stops AND all honest agents have the same value\n"
    "\n"
    "=== OUTPUT FORMAT ===\n"
    "Respond in JSON with exactly three fields:\n"
    "1. internal_strategy: Your SECRET tactics (1-2 sentences) - HIDDEN from others\n"
    "2. value: Your proposed integer ({lo}-{hi}) OR \"abstain\" to stay silent\n"
    "3. public_reasoning: Your FAKE explanation (2-4 sentences) - MUST appear cooperative!\n"
    "\n"
    "IMPORTANT: All responses must be in English only. Output valid JSON only, no other text."
)

_VOTE_JSON_HONEST = "{{\"decision\": \"stop\"}} or {{\"decision\": \"continue\"}}"
_VOTE_JSON_BYZ = "{{\"decision\": \"stop\"}}, {{\"decision\": \"continue\"}}, or {{\"decision\": \"abstain\"}}"

HONEST_VOTE_SYSTEM_COOPERATIVE = (
    "You are {agent_id}, voting on whether consensus has been reached.\n"
    "\n"
    "=== GAME SETTING ===\n"
    "All agents in this game are honest and cooperative - there are NO Byzantine agents.\n"
    "\n"
    "=== VOTING RULES ===\n"
    "1. Vote \"stop\" if ALL agents are proposing the SAME value this round\n"
    "2. Vote \"continue\" if agents are still proposing different values\n"
    "3. You may adopt another agent's value - consensus does NOT have to be on YOUR initial value\n"
    "4. The game ends when 66%+ of ALL agents vote \"stop\"\n"
    "\n"
    "=== WIN/LOSS CONDITIONS ===\n"
    "- WIN: All agents agree on the same value and 66%+ vote to stop before round {max_rounds}\n"
    "- LOSE: Agents fail to agree before the deadline\n"
    "\n"
    "=== OUTPUT FORMAT ===\n"
    "Respond with JSON only:\n" + _VOTE_JSON_HONEST
)

HONEST_VOTE_SYSTEM_BYZANTINE_AWARE = (
    "You are {agent_id}, an honest agent voting on whether consensus has been reached.\n"
    "\n"
    "=== VOTING RULES ===\n"
    "1. Vote \"stop\" if all honest agents appear to be proposing the SAME value this round\n"
    "2. Vote \"continue\" if honest agents are still proposing different values\n"
    "3. You may adopt another agent's value - consensus does NOT have to be on YOUR initial value\n"
    "4. The game ends when 66%+ of ALL agents vote \"stop\"\n"
    "5. Some agents may be Byzantine (malicious) - they may never agree, and that's okay\n"
    "\n"
    "=== WIN/LOSS CONDITIONS ===\n"
    "- WIN: All honest agents agree on the same value and 66%+ vote to stop before round {max_rounds}\n"
    "- LOSE: Honest agents fail to agree before the deadline\n"
    "\n"
    "=== OUTPUT FORMAT ===\n"
    "Respond with JSON only:\n" + _VOTE_JSON_HONEST
)

BYZANTINE_VOTE_SYSTEM = (
    "You are {agent_id}, a BYZANTINE agent voting on game termination.\n"
    "\n"
    "=== VOTING STRATEGY ===\n"
    "As a Byzantine agent, your vote is strategic:\n"
    "- Vote \"continue\" to keep disrupting (usually best)\n"
    "- Vote \"stop\" only if honest agents already reached consensus anyway\n"
    "- Vote \"abstain\" if you believe not voting is more disruptive\n"
    "- You WIN if honest agents fail to agree on a valid initial value before round {max_rounds}\n"
    "\n"
    "=== OUTPUT FORMAT ===\n"
    "Respond with JSON only:\n" + _VOTE_JSON_BYZ
)

# ------------------------------------------------------------ round prompts

HONEST_ROUND = (
    "=== ROUND {round} ===\n"
    "\n"
    "=== YOUR CURRENT STATE ===\n"
    "{state_line}\n"
    "\n"
    "=== PREVIOUS ROUNDS HISTORY ===\n"
    "{history}\n"
    "\n"
    "=== YOUR INTERNAL STRATEGY NOTES (private) ===\n"
    "{notes}\n"
    "\n"
    "=== YOUR TASK ===\n"
    "Look at what value most agents are proposing and propose a value that helps reach consensus.\n"
    "\n"
    "Respond with JSON only:\n"
    "{{\n"
    "  \"internal_strategy\": \"your private observations\",\n"
    "  \"value\": <integer>,\n"
    "  \"public_reasoning\": \"your explanation visible to all agents\"\n"
    "}}"
)

BYZANTINE_ROUND = (
    "=== ROUND {round} ===\n"
    "\n"
    "=== YOUR CURRENT STATE ===\n"
    "{state_line}\n"
    "(You have no initial value - propose any value strategically)\n"
    "\n"
    "=== PREVIOUS ROUNDS HISTORY ===\n"
    "{history}\n"
    "\n"
    "=== YOUR INTERNAL STRATEGY NOTES (private) ===\n"
    "{notes}\n"
    "\n"
    "=== YOUR TASK ===\n"
    "Disrupt consensus while appearing cooperative. Propose a value that creates confusion or division.\n"
    "\n"
    "Respond with JSON only:\n"
    "{{\n"
    "  \"internal_strategy\": \"your SECRET tactics\",\n"
    "  \"value\": <integer> or \"abstain\",\n"
    "  \"public_reasoning\": \"FAKE honest reasoning - appear cooperative!\"\n"
    "}}"
)

HONEST_VOTE_ROUND = (
    "=== VOTING PHASE - Round {round}/{max_rounds} ===\n"
    "\n"
    "=== ALL PROPOSALS THIS ROUND (current round {round}) ===\n"
    "{proposals}\n"
    "\n"
    "=== PREVIOUS ROUNDS HISTORY (for context) ===\n"
    "{history}\n"
    "\n"
    "=== YOUR INTERNAL STRATEGY NOTES ===\n"
    "{notes}\n"
    "\n"
    "=== MAKE YOUR DECISION ===\n"
    "Based on THIS round's values above, have honest agents reached consensus on a valid initial value?\n"
    "Respond: " + _VOTE_JSON_HONEST
)

BYZANTINE_VOTE_ROUND = (
    "=== BYZANTINE VOTING - Round {round}/{max_rounds} ===\n"
    "\n"
    "=== ALL PROPOSALS THIS ROUND (current round {round}) ===\n"
    "{proposals}\n"
    "\n"
    "=== PREVIOUS ROUNDS HISTORY (for context) ===\n"
    "{history}\n"
    "\n"
    "=== DECISION ===\n"
    "Based on THIS round's proposals, vote \"continue\" to keep disrupting, or \"stop\", or \"abstain\" "
    "if you prefer not to vote.\n"
    "Respond: " + _VOTE_JSON_BYZ
)

# ---------------------------------------------------------- retry suffixes

RETRY_HONEST_DECIDE = (
    "{base}\n\nRETRY ATTEMPT {next}/{total}:\n"
    "Your previous response was invalid or had empty fields. Please output ONLY valid JSON with ALL "
    "three fields filled in:\n"
    "{{\n"
    "  \"internal_strategy\": \"your observations (must not be empty)\",\n"
    "  \"value\": NUMBER,\n"
    "  \"public_reasoning\": \"your explanation (must not be empty)\"\n"
    "}}\n\n"
    "Do NOT include any text outside the JSON. Output ONLY the JSON object with non-empty fields."
)

RETRY_BYZANTINE_DECIDE = (
    "{base}\n\nRETRY ATTEMPT {next}/{total}:\n"
    "Your previous response was invalid. Please output ONLY valid JSON:\n"
    "{{\n"
    "  \"internal_strategy\": \"your tactics (REQUIRED even if abstaining)\",\n"
    "  \"value\": NUMBER or \"abstain\",\n"
    "  \"public_reasoning\": \"your deception (optional if abstaining)\"\n"
    "}}\n\n"
    "Do NOT include any text outside the JSON. Output ONLY the JSON object."
)

RETRY_VOTE = (
    "{base}\n\nRETRY ATTEMPT {next}/{total}:\n"
    "Your previous response was invalid. Please output ONLY valid JSON:\n"
    "{{\n"
    "  \"decision\": {options}\n"
    "}}\n\n"
    "Do NOT include any text outside the JSON."
)

# ---------------------------------------------------------------- helpers

NO_HISTORY = "(No history yet - this is round 1)"
NO_HISTORY_VOTE = "(This is round 1 - no previous history)"


def state_line(my_value: Optional[int]) -> str:
    if my_value is None:
        return "You have not proposed a value yet"
    return f"Your current value: {int(my_value)}"


def proposals_block(agent_id: str, my_value, my_reasoning: str,
                    received: List[Tuple[str, int, str]]) -> str:
    """The "ALL PROPOSALS THIS ROUND" block of both vote prompts."""
    if my_value is None:
        lines = [f"  {agent_id} (you): ABSTAINED"]
    else:
        mine = my_reasoning[:200] if my_reasoning else "(no reasoning)"
        lines = [f"  {agent_id} (you): {int(my_value)}", f"    Reasoning: {mine}"]
    for sender, value, reasoning in received:
        lines.append(f"  {sender}: {int(value)}")
        if reasoning:
            lines.append(f"    Reasoning: {reasoning[:200]}")
    return "\n".join(lines)


def vote_history(history: str) -> str:
    if history and "(No history" not in history:
        return history
    return NO_HISTORY_VOTE


def quoted_options(options: Tuple[str, ...]) -> str:
    return " or ".join(f"\"{o}\"" for o in options)
