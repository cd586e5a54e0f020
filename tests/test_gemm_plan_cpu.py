"""GEMM dispatch plan (ops/gemm_plan.py) on the CPU: table lookups, the 256x256 kernel's
shape rules, and the no-library mode the overlapped-prefill engine relies on."""
import json

from byzantine_consensus_llm_agents_amd.ops.gemm_plan import PP_CFG, GemmPlan


def _plan(tmp_path, choice, timings):
    path = tmp_path / "t.json"
    path.write_text(json.dumps({"choice": choice, "timings_us": timings}))
    return GemmPlan(lib=None, table=str(path))


def test_table_and_nearest_bucket(tmp_path, monkeypatch):
    monkeypatch.setenv("BCG_HAND_GEMM", "1")
    p = _plan(tmp_path, {"448,5120,5120,2": [9, 1], "768,5120,5120,2": [-1, 1], "16384,34816,5120,1": [10, 1]},
              {})
    assert p.choose(448, 5120, 5120, 2) == (9, 1)
    assert p.choose(430, 5120, 5120, 2) == (9, 1)          # nearest measured M above
    assert p.choose(700, 5120, 5120, 2) is None             # library measured faster
    assert p.choose(9000, 34816, 5120, 1) == (PP_CFG, 1)    # prefill chunk -> 16384 entry
    assert p.choose(20000, 34816, 5120, 1) is None          # nothing measured above: library


def test_pp_shape_rules(monkeypatch):
    monkeypatch.setenv("BCG_HAND_GEMM", "1")
    p = GemmPlan(lib=None, table=None)
    assert p.supported(PP_CFG, 768, 151936, 5120, 0)       # LM head: N = 593.5 tiles, masked tail
    assert not p.supported(PP_CFG, 768, 151930, 5120, 0)   # N % 16
    assert not p.supported(PP_CFG, 768, 1000, 5120, 1)     # silu: inter % 128
    assert p.supported(PP_CFG, 768, 2 * 17408, 5120, 1)
    assert not p.supported(PP_CFG, 300000, 8192, 8192, 0)  # X beyond 4 GiB (32-bit buffer offsets)
    assert not p.supported(PP_CFG, 64, 256, 100, 0)        # K % 64


def test_fp8_plan_table_rule_and_library(tmp_path, monkeypatch):
    """fp8 projections: measured shapes follow the table (nearest M above, library beyond the
    largest measured M or where it won), unmeasured shapes the hand kernel up to M = 128."""
    from byzantine_consensus_llm_agents_amd.ops.gemm_plan import FP8_TABLE, TILES, Fp8Plan
    monkeypatch.setenv("BCG_HAND_GEMM", "1")
    path = tmp_path / "f8.json"
    path.write_text(json.dumps({"choice": {"64,8192,6144": [5, 2], "256,8192,6144": [9, 2],
                                           "320,8192,6144": [-1, 1]}}))
    tiles = dict(enumerate(TILES))
    p = Fp8Plan(tiles, str(path))
    assert p.choose(40, 8192, 6144) == (5, 2)
    assert p.choose(200, 8192, 6144) == (9, 2)
    assert p.choose(300, 8192, 6144) is None       # library measured faster
    assert p.choose(600, 8192, 6144) is None       # beyond the measured range
    assert p.choose(100, 4096, 6144) == (0, 1)     # unmeasured shape: rule
    assert p.choose(16, 4096, 6144) == (6, 1)
    assert p.choose(200, 4096, 6144) is None
    assert p.choose(64, 4096, 6100) is None        # K % 128
    monkeypatch.setenv("BCG_HAND_GEMM", "0")
    assert p.choose(40, 8192, 6144) is None
    monkeypatch.setenv("BCG_HAND_GEMM", "1")
    shipped = Fp8Plan(tiles, FP8_TABLE)            # the shipped Mistral-22B table loads and is usable
    assert shipped.table and shipped.choose(160, 8192, 6144) is not None


def test_store_epilogue_takes_residual_table_entry():
    """TP row-parallel o / down projections are called with the store epilogue (the residual
    add rides in the fused all-reduce) but the table measured them with the residual epilogue:
    the same tile loop, so the plan takes that choice."""
    from byzantine_consensus_llm_agents_amd.ops.gemm_plan import GemmPlan
    plan = GemmPlan()
    for M in (16, 256, 704):
        for N, K in ((5120, 2048), (5120, 6400)):  # Qwen3-32B TP=4 o / down shards
            assert plan._lookup(M, N, K, 0) is None and plan._lookup(M, N, K, 2) is not None
            got = plan.choose(M, N, K, 0)
            want = plan.choose(M, N, K, 2)
            assert got == want
