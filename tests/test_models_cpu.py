"""Model numerics on CPU: HF transformers parity, checkpoint IO, tensor parallelism (gloo, 2 ranks)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from byzantine_consensus_llm_agents_amd.models.batch import alloc_kv, prefill_batch
from byzantine_consensus_llm_agents_amd.models.config import get_model_config
from byzantine_consensus_llm_agents_amd.models.loader import load_safetensors_dir, save_hf_checkpoint
from byzantine_consensus_llm_agents_amd.models.transformer import DecoderModel, TPGroup
from byzantine_consensus_llm_agents_amd.ops import get_ops

SEQS = [[5, 17, 99, 1000, 7, 7, 42] * 5, [3, 1, 4, 1, 5, 9, 2, 6, 5, 3, 5], list(range(100, 160))]


def _model(name, tp=None, seed=1):
    cfg = get_model_config(name)
    m = DecoderModel(cfg, get_ops("torch"), "cpu", torch.float32, tp)
    m.init_random(seed=seed, std=0.05)
    return m


def _forward(m, seqs=SEQS):
    tokens, meta, nblk = prefill_batch(seqs)
    k, v = alloc_kv(m, nblk)
    return m.forward(tokens, meta, k, v)


@pytest.mark.parametrize("name,hf_cls", [("bcg/tiny-qwen3", "Qwen3ForCausalLM"),
                                         ("bcg/tiny-qwen2", "Qwen2ForCausalLM"),
                                         ("bcg/tiny-mistral", "MistralForCausalLM")])
def test_matches_hf_transformers(name, hf_cls, tmp_path):
    """Last-token logits of the paged engine model == HF transformers' eager forward (parity pinned)."""
    import transformers
    from byzantine_consensus_llm_agents_amd.models.loader import hf_config_dict
    m = _model(name)
    ours = _forward(m)
    cfg_d = hf_config_dict(m.cfg)
    cfg_d.pop("torch_dtype")
    arch_cfg = {"Qwen3ForCausalLM": transformers.Qwen3Config, "Qwen2ForCausalLM": transformers.Qwen2Config,
                "MistralForCausalLM": transformers.MistralConfig}[hf_cls]
    hf_cfg = arch_cfg(**{k: v for k, v in cfg_d.items() if k != "model_type"})
    hf_cfg._attn_implementation = "eager"
    hf = getattr(transformers, hf_cls)(hf_cfg).float().eval()
    missing, unexpected = hf.load_state_dict(m.hf_state_dict(), strict=False)
    tied = {"lm_head.weight"} if m.cfg.tie_embeddings else set()
    assert not unexpected and all("rotary" in k or k in tied for k in missing), (missing, unexpected)
    if tied:
        assert hf.lm_head.weight.data_ptr() == hf.model.embed_tokens.weight.data_ptr()
    for r, s in enumerate(SEQS):
        with torch.no_grad():
            ref = hf(torch.tensor([s])).logits[0, -1]
        torch.testing.assert_close(ours[r], ref, atol=2e-4, rtol=2e-4)


def test_checkpoint_roundtrip_sharded(tmp_path):
    m = _model("bcg/tiny-qwen2")  # QKV bias + tied embeddings
    save_hf_checkpoint(m.hf_state_dict(), m.cfg, str(tmp_path), max_shard_bytes=4 << 20)
    assert os.path.exists(tmp_path / "model.safetensors.index.json")
    cfg = get_model_config("x", str(tmp_path))
    assert cfg.qkv_bias and cfg.tie_embeddings and cfg.num_layers == m.cfg.num_layers
    m2 = DecoderModel(cfg, get_ops("torch"), "cpu", torch.float32)
    m2.load_hf_state_dict(load_safetensors_dir(str(tmp_path)))
    torch.testing.assert_close(_forward(m2), _forward(m), atol=0, rtol=0)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _tp_worker(rank, world, port, ckpt, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from byzantine_consensus_llm_agents_amd.parallel import groups
    groups.init_distributed("gloo")
    tp = groups.tensor_parallel_group(world)
    cfg = get_model_config("x", ckpt)
    m = DecoderModel(cfg, get_ops("torch"), "cpu", torch.float32, tp)
    m.load_hf_state_dict(load_safetensors_dir(ckpt))
    logits = _forward(m)
    if rank == 0:
        torch.save(logits, out)
    groups.destroy()


def test_tensor_parallel_2_ranks_matches_tp1(tmp_path):
    m = _model("bcg/tiny-qwen3")
    ckpt = str(tmp_path / "ckpt")
    save_hf_checkpoint(m.hf_state_dict(), m.cfg, ckpt)
    out = str(tmp_path / "logits.pt")
    mp.start_processes(_tp_worker, args=(2, _free_port(), ckpt, out), nprocs=2, join=True, start_method="spawn")
    got = torch.load(out, weights_only=True)
    torch.testing.assert_close(got, _forward(m), atol=1e-4, rtol=1e-4)


def test_tp_group_identity_without_distributed():
    g = TPGroup()
    x = torch.ones(3, 4)
    assert g.all_reduce_(x) is x and g.all_gather_last(x) is x


def _engine_tp_worker(rank, world, port, ckpt, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import json
    from byzantine_consensus_llm_agents_amd.parallel import groups
    groups.init_distributed("gloo")
    texts = _engine_texts(ckpt, tp=world, seed=None if rank else 11, async_=os.environ.get("TP_ASYNC","1")=="1" and rank == 0)  # rank 0's seed wins
    with open(f"{out}.{rank}", "w") as fh:
        json.dump(texts, fh)
    groups.destroy()


def _engine_texts(ckpt, tp, seed, async_=False):
    """Rank 0 (driver) serves two generate() calls; a TP follower replays its plans."""
    from byzantine_consensus_llm_agents_amd.bcg import prompts as P
    from byzantine_consensus_llm_agents_amd.engine import GuidedDecodingParams, LLM, SamplingParams
    llm = LLM("bcg/tiny-qwen3", backend="torch", weights=ckpt, tensor_parallel_size=tp, seed=seed,
              max_model_len=512, kv_cache_gb=0.05, max_batch_seqs=8, dtype=torch.float32,
              budget_aware_json=True)
    if not llm.is_driver:
        llm.serve_worker()
        llm.shutdown()
        return None
    if async_:
        llm.start_continuous_batching()  # the driver keeps iteration-level batching under TP
    schemas = [P.honest_decision_schema(0, 50), P.vote_schema(P.BYZANTINE_VOTE_OPTIONS)]
    texts = []
    for call in range(2):
        prompts = [f"<|im_start|>user\nagent_{i} proposes {i * 7 + call}<|im_end|>\n<|im_start|>assistant\n"
                   for i in range(6)]
        params = [SamplingParams(temperature=[0.0, 0.5][i % 2], max_tokens=48,
                                 guided_decoding=GuidedDecodingParams(json=schemas[i % 2])) for i in range(6)]
        texts += [o.outputs[0].text for o in llm.generate(prompts, params)]
    llm.shutdown()
    return texts


def test_engine_tensor_parallel_driver_follower(tmp_path):
    """TP=2 (gloo): the follower replays the driver's plans; outputs equal the TP=1 engine's (same seed)."""
    import json
    m = _model("bcg/tiny-qwen3")
    ckpt = str(tmp_path / "ckpt")
    save_hf_checkpoint(m.hf_state_dict(), m.cfg, ckpt)
    out = str(tmp_path / "texts")
    mp.start_processes(_engine_tp_worker, args=(2, _free_port(), ckpt, out), nprocs=2, join=True,
                       start_method="spawn")
    r0, r1 = (json.load(open(f"{out}.{r}")) for r in range(2))
    assert r1 is None
    assert r0 == _engine_texts(ckpt, tp=1, seed=11)
    for t in r0:
        json.loads(t)


@pytest.mark.parametrize("name", ["bcg/tiny-mistral", "bcg/tiny-qwen3"])
def test_fp8_model_tracks_bf16(name):
    """fp8 (e4m3fn, row-wise scales) projections stay close to the unquantised model."""
    ref = _model(name)
    cfg = ref.cfg
    m8 = DecoderModel(cfg, get_ops("torch"), "cpu", torch.bfloat16, quant="fp8")
    m8.load_hf_state_dict(ref.hf_state_dict())
    assert m8.layers[0]["qkv"].dtype == torch.float8_e4m3fn and m8.layers[0]["qkv_s"].shape == (
        m8.layers[0]["qkv"].shape[0],)
    a, b = _forward(ref).float(), _forward(m8).float()
    cos = torch.nn.functional.cosine_similarity(a, b, dim=-1)
    assert cos.min() > 0.985, cos  # e4m3 (3 mantissa bits) on random-init weights
    assert (a.argmax(-1) == b.argmax(-1)).float().mean() >= 2 / 3


def test_quant_fp8_reference_roundtrip():
    from byzantine_consensus_llm_agents_amd.ops import reference as R
    x = torch.randn(7, 64) * torch.logspace(-3, 3, 7)[:, None]
    q, s = R.quant_fp8(x)
    assert q.dtype == torch.float8_e4m3fn and s.shape == (7,)
    assert (q.float().abs().amax(-1) == 448).all()
    back = q.float() * s[:, None]
    assert ((back - x).abs() <= x.abs().amax(-1, keepdim=True) / 16).all()  # e4m3: 3 mantissa bits


@pytest.mark.parametrize("name", ["bcg/tiny-qwen3", "bcg/tiny-mistral"])
def test_last_layer_row_selection_is_exact(name):
    """The last layer's o_proj / MLP run on the logits rows only (``_last_layer_rows``): the
    logits and the KV cache equal a forward that computes every row and selects afterwards."""
    import dataclasses
    m = _model(name)
    tokens, meta, nblk = prefill_batch(SEQS)
    k1, v1 = alloc_kv(m, nblk)
    sel = m.forward(tokens, meta, k1, v1)
    k2, v2 = alloc_kv(m, nblk)
    full = m.forward(tokens, dataclasses.replace(meta, logits_idx=None), k2, v2)
    assert full.shape[0] == tokens.shape[0] and sel.shape[0] == len(SEQS)
    torch.testing.assert_close(sel, full.index_select(0, meta.logits_idx), atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(k1, k2, atol=0, rtol=0)
    torch.testing.assert_close(v1, v2, atol=0, rtol=0)
