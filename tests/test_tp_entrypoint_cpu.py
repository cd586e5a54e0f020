"""Tensor parallelism from the reference's own entry point (CPU, gloo, torch ops).

The reference reaches TP through a plain ``python main.py`` run: vLLM's ``LLM``
spawns its worker processes (``bcg/vllm_agent.py:126-144``).  Here
``python -m byzantine_consensus_game.main --tp 2`` must do the same: no
torchrun, the engine spawns rank 1 itself, rank 0 drives the game and the
follower replays its schedule.  With a fixed ``--seed`` and fp32 weights the
results JSON equals the TP=1 run's (timestamp aside): same prompts, same
sampled tokens, same game.
"""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp, tp):
    work = os.path.join(tmp, f"tp{tp}")
    os.makedirs(work)
    cmd = [sys.executable, "-m", "byzantine_consensus_game.main", "--honest", "2", "--byzantine", "1",
           "--rounds", "2", "--seed", "7", "--engine", "torch", "--model", "bcg/tiny-qwen3",
           "--budget-aware-json", "--tp", str(tp)]
    env = dict(os.environ, PYTHONPATH=ROOT, BCG_DTYPE="float32", OMP_NUM_THREADS="2")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    p = subprocess.run(cmd, cwd=work, env=env, capture_output=True, text=True, timeout=900)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-4000:])
    with open(os.path.join(work, "results", "json", "run_001.json")) as fh:
        out = json.load(fh)
    out.pop("timestamp", None)
    out["metrics"].pop("timestamp", None)
    return out


@pytest.mark.slow
def test_main_tp2_spawns_worker_and_matches_tp1(tmp_path):
    one = _run(str(tmp_path), 1)
    two = _run(str(tmp_path), 2)
    assert one["rounds"] and one["statistics"]["total_rounds"] >= 1
    for key in ("statistics", "metrics", "rounds", "final_state", "a2a_message_count"):
        assert two[key] == one[key], key
