"""utils/threads.py: the per-rank host thread budget bench.py and bcg/sweep.py set before any pool
starts (the node's CPUs split over its ranks; an explicit environment wins)."""
import os

from byzantine_consensus_llm_agents_amd.utils.threads import rank_thread_budget


def test_rank_thread_budget_splits_cpus(monkeypatch):
    for k in ("RAYON_NUM_THREADS", "OMP_NUM_THREADS", "LOCAL_WORLD_SIZE"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(64)))
    assert rank_thread_budget(8) == 8
    assert os.environ["RAYON_NUM_THREADS"] == "8" and os.environ["OMP_NUM_THREADS"] == "8"


def test_rank_thread_budget_respects_explicit_env(monkeypatch):
    monkeypatch.setenv("RAYON_NUM_THREADS", "3")
    monkeypatch.delenv("OMP_NUM_THREADS", raising=False)
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "4")
    monkeypatch.setattr(os, "sched_getaffinity", lambda pid: set(range(256)))
    assert rank_thread_budget(8) == 16  # 256 / 4 local ranks, capped at 16
    assert os.environ["RAYON_NUM_THREADS"] == "3"
