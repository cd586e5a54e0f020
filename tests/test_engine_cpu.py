"""Engine on the torch backend (CPU): guided JSON, heterogeneous schemas, continuous batching."""
import json
import threading

import pytest

from byzantine_consensus_llm_agents_amd.bcg import prompts as P


@pytest.fixture(scope="module")
def llm():
    from byzantine_consensus_llm_agents_amd.bcg.config import ENGINE_CONFIG
    from byzantine_consensus_llm_agents_amd.engine import LLM
    ENGINE_CONFIG["budget_aware_json"] = True
    eng = LLM("bcg/tiny-qwen3", backend="torch", seed=3, max_model_len=1024, kv_cache_gb=0.25,
              max_batch_seqs=12)
    yield eng
    eng.shutdown()
    ENGINE_CONFIG["budget_aware_json"] = False


SCHEMAS = [P.honest_decision_schema(0, 50), P.byzantine_decision_schema(0, 50),
           P.vote_schema(P.HONEST_VOTE_OPTIONS), P.vote_schema(P.BYZANTINE_VOTE_OPTIONS)]


def _params(i, max_tokens=24):
    """Decide schemas need ~15+ tokens for their shortest JSON, votes ~6."""
    from byzantine_consensus_llm_agents_amd.engine import GuidedDecodingParams, SamplingParams
    if i % 4 < 2:
        max_tokens += 32
    return SamplingParams(temperature=[0.0, 0.5][i % 2], max_tokens=max_tokens,
                          guided_decoding=GuidedDecodingParams(json=SCHEMAS[i % 4]))


def _check(outs, params):
    for o, p in zip(outs, params):
        obj = json.loads(o.outputs[0].text)
        sch = p.guided_decoding.json
        assert set(sch["required"]) <= set(obj) <= set(sch["properties"])


def test_sync_heterogeneous_batch(llm):
    prompts = [f"<|im_start|>user\nagent_{i} round {i}<|im_end|>\n<|im_start|>assistant\n" for i in range(8)]
    params = [_params(i) for i in range(8)]
    outs = llm.generate(prompts, params)
    _check(outs, params)
    assert llm.backend.stats["calls"] >= 1


def test_more_requests_than_rows_and_prefix_cache(llm):
    # 20 sequences through 12 rows: admission waits for rows, compaction reuses them
    base = "<|im_start|>system\n" + "You are a careful consensus agent. " * 8 + "<|im_end|>\n"
    prompts = [base + f"<|im_start|>user\nround {i}<|im_end|>\n<|im_start|>assistant\n" for i in range(20)]
    params = [_params(i, max_tokens=[8, 24, 16][i % 3]) for i in range(20)]
    before = llm.backend.stats["cached_tokens"]
    _check(llm.generate(prompts, params), params)
    _check(llm.generate(prompts[:4], params[:4]), params[:4])
    assert llm.backend.stats["cached_tokens"] > before


def test_continuous_batching_threads(llm):
    llm.start_continuous_batching()
    results = {}

    def client(k):
        prompts = [f"<|im_start|>user\nclient {k} msg {j}<|im_end|>\n<|im_start|>assistant\n" for j in range(3)]
        params = [_params(k + j, max_tokens=8 + 4 * j) for j in range(3)]
        results[k] = (llm.generate(prompts, params), params)

    threads = [threading.Thread(target=client, args=(k,)) for k in range(5)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=600)
    assert len(results) == 5
    for outs, params in results.values():
        _check(outs, params)


def test_chunked_prefill_matches_single_chunk(llm):
    """Prompts straddling prefill chunks (odd chunk size) give the same greedy outputs."""
    from byzantine_consensus_llm_agents_amd.engine import GuidedDecodingParams, SamplingParams
    eng = llm.backend
    prompts = [f"<|im_start|>system\nagent {i} " + "long history entry. " * (6 + 5 * i)
               + "<|im_end|>\n<|im_start|>assistant\n" for i in range(4)]
    params = [SamplingParams(temperature=0.0, max_tokens=40,
                             guided_decoding=GuidedDecodingParams(json=SCHEMAS[i % 4])) for i in range(4)]
    saved = (eng.args.prefill_chunk_tokens, eng.args.prefix_caching)
    try:
        eng.args.prefix_caching = False
        eng.args.prefill_chunk_tokens = 1 << 14
        ref = [o.outputs[0].text for o in llm.generate(prompts, params)]
        eng.args.prefill_chunk_tokens = 37
        chunks0 = eng.stats["prefill_chunks"]
        got = [o.outputs[0].text for o in llm.generate(prompts, params)]
        assert eng.stats["prefill_chunks"] - chunks0 > 4
    finally:
        eng.args.prefill_chunk_tokens, eng.args.prefix_caching = saved
    assert got == ref


def test_engine_fp8_kv_cache_cpu(fresh_engine_state):
    """kv_cache_dtype=fp8: e4m3fn caches end to end on the reference ops; guided JSON stays valid."""
    import json
    import torch
    from byzantine_consensus_llm_agents_amd.bcg import prompts as P
    from byzantine_consensus_llm_agents_amd.engine import GuidedDecodingParams, LLM, SamplingParams
    llm = LLM("bcg/tiny-qwen3", backend="torch", seed=3, max_model_len=512, kv_cache_gb=0.02,
              max_batch_seqs=8, budget_aware_json=True, kv_cache_dtype="fp8")
    assert llm.backend.k_cache.dtype == torch.float8_e4m3fn
    params = [SamplingParams(temperature=0.5, max_tokens=40,
                             guided_decoding=GuidedDecodingParams(json=P.honest_decision_schema(0, 50)))] * 3
    outs = llm.generate([f"<|im_start|>user\nagent_{i}<|im_end|>\n<|im_start|>assistant\n" for i in range(3)],
                        params)
    for o in outs:
        assert "value" in json.loads(o.outputs[0].text)
    assert llm.backend.k_cache.float().abs().sum() > 0
    llm.shutdown()


def test_engine_admission_batching_cpu(fresh_engine_state):
    """Deferred admission (prompts queue while others decode) still completes every request."""
    import json
    import threading
    from byzantine_consensus_llm_agents_amd.bcg import prompts as P
    from byzantine_consensus_llm_agents_amd.engine import GuidedDecodingParams, LLM, SamplingParams
    llm = LLM("bcg/tiny-qwen3", backend="torch", seed=4, max_model_len=512, kv_cache_gb=0.05,
              max_batch_seqs=16, budget_aware_json=True, admit_max_wait=3, admit_min_live=1,
              prefill_chunk_tokens=4096)
    assert llm.backend.args.admit_max_wait == 3
    llm.start_continuous_batching()
    schema = P.vote_schema(P.HONEST_VOTE_OPTIONS)
    results, errors = [], []

    def client(k):
        try:
            for rnd in range(2):
                params = [SamplingParams(temperature=0.5, max_tokens=12 + 4 * k,
                                         guided_decoding=GuidedDecodingParams(json=schema))] * 2
                outs = llm.generate([f"<|im_start|>user\nc{k} r{rnd} {j}<|im_end|>\n<|im_start|>assistant\n"
                                     for j in range(2)], params)
                results.extend(json.loads(o.outputs[0].text)["decision"] for o in outs)
        except BaseException as exc:
            errors.append(exc)

    threads = [threading.Thread(target=client, args=(k,)) for k in range(4)]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=300)
    llm.shutdown()
    assert not errors, errors[0]
    assert len(results) == 16 and set(results) <= {"stop", "continue"}


def test_synthetic_tokenizer_is_pinned(monkeypatch):
    """The shipped synthetic tokenizers match their pinned SHA-256 (same token ids on every
    box, whatever its site-packages); a file with another hash is refused."""
    import hashlib

    from byzantine_consensus_llm_agents_amd.engine import tokenizer as T
    for fam in ("qwen", "mistral"):
        assert hashlib.sha256(T.synthetic_json(fam).encode()).hexdigest() == T.PINNED_SHA256[fam]
    monkeypatch.setitem(T.PINNED_SHA256, "mistral", "0" * 64)
    monkeypatch.delenv("BCG_ALLOW_UNPINNED_TOKENIZER", raising=False)
    with pytest.raises(RuntimeError, match="pinned"):
        T.synthetic_json("mistral")


def test_decode_buckets_cover_every_batch_size():
    """Every decode batch size up to the largest bucket maps to the smallest bucket >= it;
    32-row steps up to 1024 rows (GEMM padding <= 31 rows), 64-row steps beyond."""
    from byzantine_consensus_llm_agents_amd.engine.graphs import BUCKETS, MAX_ROWS, bucket_for
    assert list(BUCKETS) == sorted(set(BUCKETS)) and MAX_ROWS == BUCKETS[-1] == 1536
    for n in range(1, MAX_ROWS + 1):
        b = bucket_for(n)
        assert b >= n and all(x < n for x in BUCKETS if x < b)
        if 160 < n <= 1024:
            assert b - n < 32
        elif n > 1024:
            assert b - n < 64


def test_prefill_carry_matches_reference(fresh_engine_state):
    """Carry-over chunked prefill (prefill_carry_bursts > 0): while rows decode, a wave's
    partial last chunk is held and its prompts finish in a later wave.  Greedy outputs equal
    those of an engine that runs every tail chunk at once, and every request completes."""
    import threading
    from byzantine_consensus_llm_agents_amd.bcg import prompts as P
    from byzantine_consensus_llm_agents_amd.engine import GuidedDecodingParams, LLM, SamplingParams
    schema = P.honest_decision_schema(0, 50)
    prompts = {(k, rnd): f"<|im_start|>system\nagent {k} " + "history line. " * (3 + 2 * k + rnd)
               + f"<|im_end|>\n<|im_start|>user\nround {rnd}<|im_end|>\n<|im_start|>assistant\n"
               for k in range(6) for rnd in range(3)}
    params = SamplingParams(temperature=0.0, max_tokens=40, guided_decoding=GuidedDecodingParams(json=schema))

    def run(carry):
        llm = LLM("bcg/tiny-qwen3", backend="torch", seed=5, max_model_len=1024, kv_cache_gb=0.05,
                  max_batch_seqs=16, budget_aware_json=True, admit_max_wait=0, admit_min_live=1,
                  prefill_chunk_tokens=96, prefill_carry_bursts=carry, prefix_caching=False)
        llm.start_continuous_batching()
        out, errors = {}, []

        def client(k):
            try:
                for rnd in range(3):
                    out[(k, rnd)] = llm.generate([prompts[(k, rnd)]], [params])[0].outputs[0].text
            except BaseException as exc:
                errors.append(exc)

        threads = [threading.Thread(target=client, args=(k,)) for k in range(6)]
        for t in threads:
            t.start()
        for t in threads:
            t.join(timeout=300)
        stats = dict(llm.backend.stats)
        llm.shutdown()
        assert not errors, errors[0]
        return out, stats

    ref, _ = run(0)
    got, stats = run(4)
    assert len(got) == 18 and got == ref
    assert stats["prefill_carried"] > 0 and stats["prefill_full_chunks"] > 0


def test_validity_aware_grammar_outputs_pass_simulator_rules(fresh_engine_state):
    """The bench grammar on the real engine (torch ops, random tiny Qwen3, budget-aware
    sampling): every decide output passes the simulator's batched validity rule -- none would
    go down the retry ladder -- and every vote is in its enum."""
    import json
    from byzantine_consensus_llm_agents_amd.bcg import prompts as P
    from byzantine_consensus_llm_agents_amd.bcg.simulation import is_valid_decision, is_valid_vote
    from byzantine_consensus_llm_agents_amd.engine import GuidedDecodingParams, LLM, SamplingParams
    llm = LLM("bcg/tiny-qwen3", backend="torch", seed=11, max_model_len=1024, kv_cache_gb=0.05,
              max_batch_seqs=16, budget_aware_json=True, validity_aware_json=10)
    schemas = [P.honest_decision_schema(0, 50), P.byzantine_decision_schema(0, 50),
               P.vote_schema(P.HONEST_VOTE_OPTIONS)]
    params = [SamplingParams(temperature=1.0, max_tokens=[150, 150, 40][i % 3],
                             guided_decoding=GuidedDecodingParams(json=schemas[i % 3])) for i in range(15)]
    outs = llm.generate([f"<|im_start|>user\nagent_{i} round 2<|im_end|>\n<|im_start|>assistant\n"
                         for i in range(15)], params)
    llm.shutdown()
    for i, o in enumerate(outs):
        obj = json.loads(o.outputs[0].text)
        assert is_valid_vote(obj) if i % 3 == 2 else is_valid_decision(obj), obj


def test_ascii_text_grammar_and_context_counters(fresh_engine_state):
    """VERDICT r5 item 2.  The ASCII bench grammar: every free-text character the random model
    writes is printable ASCII (no escapes / multi-byte UTF-8 that re-tokenise at several tokens per
    character in later prompts).  A prompt at the context limit is answered "" and counted
    (context_rejects); one whose context room is below the grammar's shortest output is counted
    (context_short); prompt sizes are recorded per requested max_tokens."""
    import json
    from byzantine_consensus_llm_agents_amd.bcg import prompts as P
    from byzantine_consensus_llm_agents_amd.bcg.simulation import is_valid_decision
    from byzantine_consensus_llm_agents_amd.engine import GuidedDecodingParams, LLM, SamplingParams
    llm = LLM("bcg/tiny-qwen3", backend="torch", seed=5, max_model_len=256, kv_cache_gb=0.05,
              max_batch_seqs=16, budget_aware_json=True, validity_aware_json=10, ascii_text_json=True)
    eng = llm.backend
    sch = P.honest_decision_schema(0, 50)
    ok = SamplingParams(temperature=1.0, max_tokens=120, guided_decoding=GuidedDecodingParams(json=sch))
    outs = llm.generate([f"<|im_start|>user\nagent_{i}<|im_end|>\n<|im_start|>assistant\n" for i in range(6)],
                        [ok] * 6)
    for o in outs:
        obj = json.loads(o.outputs[0].text)
        assert is_valid_decision(obj), obj
        for field in ("internal_strategy", "public_reasoning"):
            assert all(0x20 <= ord(c) <= 0x7E for c in obj[field]), obj[field]
    n_tok = lambda s: len(eng.tokenizer.encode(s))  # noqa: E731
    filler = "word " * 400
    long_p = filler[:len(filler)]
    while n_tok(long_p) > 300:
        long_p = long_p[:-50]
    assert n_tok(long_p) >= 256
    near = long_p
    while n_tok(near) > 250:  # 6 tokens of room: below the decide grammar's shortest output
        near = near[:-5]
    outs = llm.generate([long_p, near], [ok, ok])
    llm.shutdown()
    assert outs[0].outputs[0].text == ""
    assert eng.stats["context_rejects"] == 1 and eng.stats["context_short"] == 1
    assert len(eng.prompt_lens[120]) == 8 and max(eng.prompt_lens[120]) == n_tok(long_p)


def test_finished_rows_skip_attention_same_outputs(fresh_engine_state, monkeypatch):
    """Rows that finished idle in the decode batch until reaped; their attention reads one token
    (engine.decode_meta attn_seq_lens) instead of the whole context.  Greedy outputs are identical
    with and without the skip (the sampler ignores finished rows), rows finishing at different steps."""
    from byzantine_consensus_llm_agents_amd.bcg import prompts as P
    from byzantine_consensus_llm_agents_amd.engine import GuidedDecodingParams, LLM, SamplingParams
    schemas = [P.honest_decision_schema(0, 50), P.vote_schema(P.HONEST_VOTE_OPTIONS)]
    prompts = [f"<|im_start|>user\nagent_{i} round 3 " + "history " * (5 * i) + "<|im_end|>\n<|im_start|>assistant\n"
               for i in range(6)]
    params = [SamplingParams(temperature=0.0, max_tokens=[70, 12, 40, 9, 55, 20][i],
                             guided_decoding=GuidedDecodingParams(json=schemas[i % 2])) for i in range(6)]
    outs = {}
    for skip in ("1", "0"):
        monkeypatch.setenv("BCG_SKIP_DONE_ATTN", skip)
        llm = LLM("bcg/tiny-qwen3", backend="torch", seed=9, max_model_len=512, kv_cache_gb=0.05,
                  max_batch_seqs=8, budget_aware_json=True)
        assert llm.backend._skip_done_attn == (skip == "1")
        outs[skip] = [o.outputs[0].text for o in llm.generate(prompts, params)]
        llm.shutdown()
    assert outs["1"] == outs["0"]


def test_prefill_tile_table_covers_rows(fresh_engine_state, monkeypatch):
    """The prefill tile table the engine builds for the HIP kernels (ops.prefill_tile_rows rows per
    tile: 128 selects the 32x32 LDS kernel): every packed query row of a chunk in exactly one tile
    of its own sequence, no tile longer than tile_rows, deepest tiles first -- checked on the torch
    backend by recording what reaches paged_attention_prefill."""
    from byzantine_consensus_llm_agents_amd.engine import LLM, SamplingParams
    from byzantine_consensus_llm_agents_amd.ops import get_ops
    ops = get_ops("torch")
    seen = []
    orig = ops.paged_attention_prefill

    def record(q, k_cache, v_cache, layer, block_tables, q_start, seq_lens, scale, max_q_len=None, tiles=None,
               tile_rows=64):
        if layer == 0:
            seen.append((tiles.cpu().tolist(), tile_rows, q_start.cpu().tolist(), seq_lens.cpu().tolist()))
        return orig(q, k_cache, v_cache, layer, block_tables, q_start, seq_lens, scale, max_q_len, tiles, tile_rows)

    monkeypatch.setattr(ops, "paged_attention_prefill", record)
    monkeypatch.setattr(ops, "prefill_tile_rows", lambda hd, kv_fp8=False, max_blocks=0: 128)
    llm = LLM("bcg/tiny-qwen3", backend="torch", seed=2, max_model_len=1024, kv_cache_gb=0.05,
              max_batch_seqs=8, prefill_chunk_tokens=256, prefix_caching=False)
    prompts = [f"<|im_start|>user\nagent_{i} " + "history " * (30 * i + 7) + "<|im_end|>\n" for i in range(5)]
    llm.generate(prompts, [SamplingParams(temperature=0.0, max_tokens=2)] * 5)
    llm.shutdown()
    assert seen
    for tiles, rows, q_start, seq_lens in seen:
        assert rows == 128
        covered = [0] * q_start[-1]
        for b, t0, t1 in tiles:
            assert q_start[b] <= t0 < t1 <= q_start[b + 1] and t1 - t0 <= rows
            for r in range(t0, t1):
                covered[r] += 1
        assert covered == [1] * q_start[-1]
        depth = [seq_lens[b] - (q_start[b + 1] - t0) for b, t0, _ in tiles]  # keys before the tile
        assert depth == sorted(depth, reverse=True)
