"""Grammar-forced decode steps of the bench FSMs: states whose budget-feasible allowed set is ONE token
(what jump-forward could skip without changing outputs), counted on random walks of the token FSM.

  python tools/forced_tokens.py
"""
import json, sys, numpy as np
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from byzantine_consensus_llm_agents_amd.engine.tokenizer import load_tokenizer
from byzantine_consensus_llm_agents_amd.engine.guided.compiler import compile_schema
from byzantine_consensus_llm_agents_amd.engine.guided.json_schema import validity_aware
from byzantine_consensus_llm_agents_amd.bcg import prompts as P
tok = load_tokenizer("Qwen/Qwen3-14B")
tb = tok.all_token_bytes()
for name, sch, budget in (("honest_decide", P.honest_decision_schema(0, 50), 300), ("byz_vote", P.vote_schema(P.BYZANTINE_VOTE_OPTIONS), 200)):
    schema = validity_aware(sch, 10, True)
    fsm = compile_schema(schema, tb, len(tb))
    nxt, dist = fsm.next, fsm.dist
    S = nxt.shape[0]
    allowed = (nxt >= 0).sum(axis=1)
    print(name, "states", S, "states with exactly 1 allowed token:", int((allowed == 1).sum()), "with <= 3:", int((allowed <= 3).sum()))
    rng = np.random.default_rng(0)
    forced_steps = tot = 0
    for trial in range(20):
        s = 0
        for step in range(budget):
            row = nxt[s]; left = budget - step - 1
            ok = np.nonzero(row >= 0)[0]; ok = ok[dist[row[ok]] <= left]
            if len(ok) == 0: break
            if len(ok) == 1: forced_steps += 1
            tot += 1
            t = int(rng.choice(ok)); s = int(row[t])
            if dist[s] == 0 and (nxt[s] >= 0).sum() == 0: break
    print("  random walk: forced steps", forced_steps, "of", tot, "(%.1f%%)" % (100*forced_steps/max(tot,1)))
