"""bench.py driver contract on CPU (gloo ranks, no GPU).

The round driver runs ``python bench.py --gpus N --steps K --warmup W`` (and
the same under torchrun) and parses exactly one JSON line from stdout.  These
tests launch it WITHOUT torchrun -- ``--gpus 2`` must start its two ranks
itself -- and check the contract: metric/value/unit, ``n_gpus``, ``steps``,
``warmup``, ``config.parallelism``; one step = one ``--window-s`` window of the
continuously running pool, ``value`` = whole-job decisions / elapsed, and the
deadline guard still prints the line with the windows actually timed.
"""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config"}


def _run(extra, timeout=300, env_extra=None):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--backend", "fake", "--sims-per-gpu", "2",
           "--honest", "4", "--byzantine", "1", "--window-s", "1"] + extra
    env = dict(os.environ, OMP_NUM_THREADS="1", **(env_extra or {}))
    env.pop("WORLD_SIZE", None)
    p = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    # gloo's C++ connection log goes to the process's stdout below Python; every JSON
    # line counts: exactly one (rank 0's) must exist
    lines = [ln for ln in p.stdout.splitlines() if ln.lstrip().startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("tp,parallelism,replicas", [(1, "dp2", 2), (2, "dp1xtp2", 1)])
def test_bench_self_launches_two_ranks(tp, parallelism, replicas):
    out = _run(["--gpus", "2", "--tp", str(tp), "--steps", "2", "--warmup", "1"])
    assert KEYS <= set(out)
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["warmup"] == 1
    assert out["unit"] == "decisions/s" and out["higher_is_better"] is True and out["scaling"] == "weak"
    assert out["config"]["parallelism"] == parallelism
    assert out["config"]["global_batch"] == 2 * 5 * replicas
    d = out["detail"]
    assert d["decisions"] > 0 and out["value"] == pytest.approx(d["decisions"] / d["elapsed_s"], rel=1e-2)
    # a step is one window: the timed region is K windows (+ the closing barrier), and it fits in
    # the process's own wall time (structural: no wall-clock upper bound on a shared box)
    assert out["ms_per_step"] >= 1000.0
    assert out["ms_per_step"] * out["steps"] <= 1000.0 * d["wall_since_start_s"]
    assert len(d["decisions_per_window_rank0"]) == 2


def test_bench_single_rank_defaults_contract():
    out = _run(["--steps", "3", "--warmup", "1"])
    assert out["n_gpus"] == 1 and out["steps"] == 3 and out["config"]["parallelism"] == "dp1"
    assert out["config"]["max_batch_seqs"] == 768 and out["config"]["sims_per_gpu"] == 2
    out = _run(["--steps", "1", "--warmup", "1", "--max-batch-seqs", "1024"])
    assert out["config"]["max_batch_seqs"] == 1024
    assert out["config"]["model"] == "Qwen/Qwen3-14B" and out["dtype"] == "bf16"
    assert out["config"]["honest"] == 4 and out["config"]["byzantine"] == 1


def test_bench_deadline_guard_reports_completed_windows():
    # 3 s of budget: the warmup window + 2 timed windows at most, never the 10 requested
    out = _run(["--steps", "10", "--warmup", "1", "--deadline-s", "3"])
    assert 1 <= out["steps"] < 10
    assert out["detail"]["steps_requested"] == 10
    assert out["ms_per_step"] * out["steps"] <= 1000.0 * out["detail"]["wall_since_start_s"]


@pytest.mark.slow
def test_bench_tp2_torch_engine_continuous_batching():
    """Real engine (torch ops, tiny Qwen3) at TP=2: the driver serves the pool with
    continuous batching, the follower replays its plans (no lock-step coalescer)."""
    out = _run(["--gpus", "2", "--tp", "2", "--backend", "torch", "--model", "bcg/tiny-qwen3",
                "--steps", "2", "--warmup", "1", "--window-s", "4"], timeout=600)
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp1xtp2" and out["steps"] == 2
    assert out["detail"]["engine_per_rank"]["decode_steps"] > 0


def test_bench_reports_resolution_fields():
    """tokens/s and the window spread are in detail, max_rounds in config."""
    out = _run(["--steps", "4", "--warmup", "1", "--max-rounds", "7"])
    d = out["detail"]
    assert out["config"]["max_rounds"] == 7
    assert {"tokens_per_s", "window_stats_rank0", "token_window_stats_rank0", "fill_max_s", "fill_capped"} <= set(d)
    assert d["window_stats_rank0"]["n"] == 4
    assert "protocol" in d["age_mix"]


def test_window_stats_block_estimate():
    sys.path.insert(0, ROOT)
    from bench import window_stats
    s = window_stats([100, 300] * 4, 12.0)  # perfectly anti-correlated neighbours
    assert s["se_pct"] > 10 and s["block4_se_pct"] == 0.0
    assert window_stats([5], 12.0) == {"n": 1}


def test_bench_hostmodel_backend_reports_host_budget():
    """--backend hostmodel: the engine's host work with a modelled GPU; detail.host carries the
    CPU seconds per decision and the slowest replica's rate."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--backend", "hostmodel", "--sims-per-gpu", "4",
           "--honest", "4", "--byzantine", "1", "--window-s", "2", "--steps", "2", "--warmup", "1"]
    env = dict(os.environ, OMP_NUM_THREADS="1", BCG_HOSTMODEL_TOKENS_S="200000")
    env.pop("WORLD_SIZE", None)
    p = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    h = out["detail"]["host"]
    assert out["detail"]["decisions"] > 0 and h["cpu_s_per_decision"] > 0
    # the timed region's prompt sizes per phase and the context-limit counters
    pt = out["detail"]["prompt_tokens_rank0"]
    assert set(pt) == {"decide", "vote"} and all(0 < v["p50"] <= v["p95"] <= v["max"] for v in pt.values())
    assert out["detail"]["context_rank0"]["rejects"] == 0
    assert out["config"]["grammar"].endswith("ascii-text")
    assert h["min_replica_decisions_per_s"] > 0 and out["detail"]["tokens_per_s"] > 0


def test_bench_reports_retry_overhead_with_fault_injector():
    """the timed region's retry-ladder cost is in detail.retry.  agent_1's
    decide requests always fail (unparsable JSON): every one of its decisions goes through the
    batch retry, the sequential 3-attempt loop, and exhausts."""
    rules = [{"agent": "agent_1", "round": r, "phase": "decide", "tries": "all", "mode": "invalid_json"}
             for r in range(1, 5)]
    out = _run(["--steps", "3", "--warmup", "1", "--age-p", "0", "--max-rounds", "4"],
               env_extra={"BCG_FAKE_FAULTS": json.dumps(rules)})
    r = out["detail"]["retry"]
    assert r["decide_prompts"] > 0 and r["vote_prompts"] > 0
    assert r["decisions_exhausted"] > 0 and r["sequential_calls"] > 0
    assert r["sequential_attempts"] >= 3 * r["decisions_exhausted"] - 3  # (a window may cut a loop)
    assert r["retry_rows"] > 0 and r["engine_rows_per_prompt"] > 1.0
    host = out["detail"]["host"]
    assert host["threads_per_rank"] >= 2 and "cpu_s_by_thread_rank0" in host


def test_bench_retry_counters_zero_without_faults():
    out = _run(["--steps", "2", "--warmup", "1", "--age-p", "0"])
    r = out["detail"]["retry"]
    assert r["decisions_exhausted"] == 0 and r["votes_exhausted"] == 0 and r["retry_rows"] >= 0


@pytest.mark.parametrize("tp,parallelism", [(4, "dp2xtp4"), (2, "dp4xtp2")])
def test_bench_world8_layouts(tp, parallelism):
    """the BASELINE layouts of configs 4 (TP=4 x DP=2) and 5 (TP=2 x DP=4) at
    world 8 (gloo ranks, scripted engine): one JSON line, one game pool per replica (its group's
    driver) with its own seeds, followers run no games, decisions summed over replicas only."""
    out = _run(["--gpus", "8", "--tp", str(tp), "--steps", "2", "--warmup", "1"], timeout=600)
    assert out["n_gpus"] == 8 and out["config"]["parallelism"] == parallelism
    replicas = 8 // tp
    assert out["config"]["global_batch"] == 2 * 5 * replicas
    ranks = sorted(out["detail"]["ranks"], key=lambda r: r["rank"])
    assert [r["rank"] for r in ranks] == list(range(8))
    assert [r["replica"] for r in ranks] == [i // tp for i in range(8)]
    drivers = [r for r in ranks if r["driver"]]
    assert [r["rank"] for r in drivers] == [tp * k for k in range(replicas)]
    assert len({r["seed_base"] for r in drivers}) == replicas and all(r["sims"] == 2 for r in drivers)
    assert all(r["decisions"] == 0 and r["sims"] == 0 for r in ranks if not r["driver"])
    assert out["detail"]["decisions"] == sum(r["decisions"] for r in drivers) > 0
