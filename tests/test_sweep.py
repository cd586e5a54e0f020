"""DP seed sweep (bcg/sweep.py): same per-seed outcomes on 1 process and on 2 gloo ranks."""
import json
import os
import socket

import torch.multiprocessing as mp

ARGS = ["--seeds", "5", "--seed0", "40", "--honest", "3", "--byzantine", "1", "--rounds", "4",
        "--engine", "fake", "--concurrency", "3"]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from byzantine_consensus_llm_agents_amd.bcg import sweep
    sweep.main(ARGS + ["--out", out])


def test_sweep_single_process(tmp_path, fresh_engine_state):
    from byzantine_consensus_llm_agents_amd.bcg import sweep
    out = str(tmp_path / "one.json")
    summary = sweep.main(ARGS + ["--out", out])
    assert summary["games"] == 5 and sum(summary["outcomes"].values()) == 5
    assert [g["seed"] for g in summary["per_game"]] == list(range(40, 45))
    assert all(g["consensus_outcome"] in sweep.OUTCOMES for g in summary["per_game"])
    assert summary["decisions"] > 0 and summary["decisions_per_s"] > 0
    on_disk = json.load(open(out))
    assert on_disk["per_game"] == summary["per_game"]


def test_sweep_two_ranks_matches_single(tmp_path, fresh_engine_state):
    from byzantine_consensus_llm_agents_amd.bcg import sweep
    single = sweep.main(ARGS + ["--out", str(tmp_path / "one.json")])
    out = str(tmp_path / "two.json")
    mp.start_processes(_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    multi = json.load(open(out))
    assert multi["n_gpus"] == 2 and multi["config"]["dp"] == 2
    strip = [{k: v for k, v in g.items()} for g in single["per_game"]]
    assert multi["per_game"] == strip  # seeds split across ranks, outcomes unchanged
    assert multi["outcomes"] == single["outcomes"]


def test_sweep_resume_from_checkpoints(tmp_path, fresh_engine_state):
    from byzantine_consensus_llm_agents_amd.bcg import sweep
    out = str(tmp_path / "res.json")
    full = sweep.main(ARGS + ["--out", out])
    ck = sweep.checkpoint_path(out, 0)
    lines = open(ck).read().splitlines()
    assert len(lines) == 5
    # simulate a run killed after two games (plus a torn line)
    with open(ck, "w") as fh:
        fh.write("\n".join(lines[:2]) + "\n" + lines[2][:10])
    resumed = sweep.main(ARGS + ["--out", out, "--resume"])
    assert resumed["resumed_games"] == 2
    assert resumed["per_game"] == full["per_game"]
    assert resumed["outcomes"] == full["outcomes"]
    assert sweep.load_checkpoints(out).keys() == {g["seed"] for g in full["per_game"]}


def _lb_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), BCG_FAKE_DELAY_S="0.004")
    from byzantine_consensus_llm_agents_amd.bcg import sweep
    sweep.main(["--seeds", "64", "--seed0", "100", "--honest", "3", "--byzantine", "1", "--rounds", "8",
                "--engine", "fake", "--concurrency", "1", "--out", out])


def test_sweep_dynamic_seed_queue_balances_replicas(tmp_path):
    """Uneven game lengths (1-8 rounds): replicas pull seeds from a shared counter,
    every seed is played exactly once, and no replica idles long at the tail."""
    out = str(tmp_path / "lb.json")
    mp.start_processes(_lb_worker, args=(2, _free_port(), out), nprocs=2, join=True, start_method="spawn")
    res = json.load(open(out))
    assert [g["seed"] for g in res["per_game"]] == list(range(100, 164))
    rounds = [g["total_rounds"] for g in res["per_game"]]
    assert max(rounds) > min(rounds)  # the games really are uneven
    assert res["replica_idle_tail_frac"] < 0.05, res["replica_idle_tail_frac"]
