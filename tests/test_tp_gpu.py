"""Tensor parallelism on the GPU path, rehearsed on a one-GPU box.

Two processes share cuda:0 (RCCL refuses two ranks on one device, so the
process group is gloo) and run the HIP kernels on TP-sharded weights; the
decode-sized all-reduces go through the custom xGMI kernels
(``BCG_CUSTOM_AR=force``: IPC-mapped peer buffers, as across GPUs).  Checks:
* the TP=2 forward reproduces the TP=1 forward (same checkpoint) to bf16 tolerance;
* a TP=2 engine (eager decode: gloo collectives cannot be graph-captured):
  rank 0 drives, rank 1 replays its plans -- same collectives on both ranks,
  schema-valid outputs.
"""
import json
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

SEQS = [[5, 17, 99, 1000, 7, 7, 42] * 5, [3, 1, 4, 1, 5, 9, 2, 6, 5, 3, 5], list(range(100, 170))]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _forward(ckpt, tp):
    from byzantine_consensus_llm_agents_amd.models.batch import alloc_kv, prefill_batch
    from byzantine_consensus_llm_agents_amd.models.config import get_model_config
    from byzantine_consensus_llm_agents_amd.models.loader import load_safetensors_dir
    from byzantine_consensus_llm_agents_amd.models.transformer import DecoderModel
    from byzantine_consensus_llm_agents_amd.ops import get_ops
    cfg = get_model_config("x", ckpt)
    m = DecoderModel(cfg, get_ops("hip"), "cuda", torch.bfloat16, tp)
    m.load_hf_state_dict(load_safetensors_dir(ckpt))
    tokens, meta, nblk = prefill_batch(SEQS, device="cuda")
    k, v = alloc_kv(m, nblk)
    return m.forward(tokens, meta, k, v).float().cpu()


def _worker(rank, world, port, ckpt, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", BCG_CUSTOM_AR="force", HSA_ENABLE_IPC_MODE_LEGACY="0")
    torch.cuda.set_device(0)
    from byzantine_consensus_llm_agents_amd.bcg import prompts as P
    from byzantine_consensus_llm_agents_amd.bcg.config import ENGINE_CONFIG
    from byzantine_consensus_llm_agents_amd.engine import GuidedDecodingParams, LLM, SamplingParams
    from byzantine_consensus_llm_agents_amd.parallel import groups
    groups.init_distributed("gloo")
    tpg = groups.tensor_parallel_group(world, custom_allreduce=True)
    assert tpg.custom is not None
    logits = _forward(ckpt, tpg)
    ENGINE_CONFIG.update(budget_aware_json=True, use_hip_graphs=False)
    llm = LLM("bcg/tiny-qwen3", backend="hip", weights=ckpt, tensor_parallel_size=world, seed=5,
              max_model_len=1024, kv_cache_gb=0.5, max_batch_seqs=16)
    schemas = [P.honest_decision_schema(0, 50), P.vote_schema(P.BYZANTINE_VOTE_OPTIONS)]
    prompts = [f"<|im_start|>user\nagent_{i} proposes {i * 7}<|im_end|>\n<|im_start|>assistant\n" for i in range(6)]
    params = [SamplingParams(temperature=[0.0, 0.5][i % 2], max_tokens=40,
                             guided_decoding=GuidedDecodingParams(json=schemas[i % 2])) for i in range(6)]
    if llm.is_driver:  # rank 0 serves; the follower replays its plans
        texts = [o.outputs[0].text for o in llm.generate(prompts, params)]
    else:
        llm.serve_worker()
        texts = None
    calls = dict(tpg.custom.calls)
    err = tpg.custom.take_error()
    llm.shutdown()
    torch.save({"logits": logits, "texts": texts, "calls": calls, "err": err}, f"{out}.{rank}")
    groups.destroy()


def test_tp2_two_processes_one_gpu(tmp_path):
    from byzantine_consensus_llm_agents_amd.models.config import get_model_config
    from byzantine_consensus_llm_agents_amd.models.loader import save_hf_checkpoint
    from byzantine_consensus_llm_agents_amd.models.transformer import DecoderModel
    from byzantine_consensus_llm_agents_amd.ops import get_ops
    cfg = get_model_config("bcg/tiny-qwen3")
    ref = DecoderModel(cfg, get_ops("torch"), "cpu", torch.bfloat16)
    ref.init_random(seed=2, std=0.05)
    ckpt = str(tmp_path / "ckpt")
    save_hf_checkpoint(ref.hf_state_dict(), cfg, ckpt)
    tp1 = _forward(ckpt, None)
    out = str(tmp_path / "tp")
    mp.start_processes(_worker, args=(2, _free_port(), ckpt, out), nprocs=2, join=True, start_method="spawn")
    r0, r1 = (torch.load(f"{out}.{r}", weights_only=True) for r in range(2))
    for r in (r0, r1):
        assert not r["err"] and r["calls"][1] > 0  # decode/prefill all-reduces took the custom kernel
        torch.testing.assert_close(r["logits"], tp1, atol=6e-2, rtol=6e-2)
    assert torch.equal(r0["logits"], r1["logits"])  # bitwise-identical activations on both ranks
    assert r0["calls"] == r1["calls"]  # the follower ran exactly the driver's collectives
    assert r1["texts"] is None
    for t in r0["texts"]:
        json.loads(t)


def _graph_worker(rank, world, port, ckpt, out, graphs):
    """TP=2 engine, decode captured in HIP graphs with the xGMI kernels inside (all-reduce,
    fused all-reduce + add + RMSNorm, logits gather) -- or eager -- then a forced all-reduce
    timeout on rank 0 that must surface as an exception, not as garbage tokens."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", BCG_CUSTOM_AR="force", HSA_ENABLE_IPC_MODE_LEGACY="0",
                      BCG_AR_TIMEOUT_S="3")
    torch.cuda.set_device(0)
    from byzantine_consensus_llm_agents_amd.bcg import prompts as P
    from byzantine_consensus_llm_agents_amd.bcg.config import ENGINE_CONFIG
    from byzantine_consensus_llm_agents_amd.engine import GuidedDecodingParams, LLM, SamplingParams
    from byzantine_consensus_llm_agents_amd.parallel import groups
    groups.init_distributed("gloo")
    ENGINE_CONFIG.update(budget_aware_json=True, use_hip_graphs=graphs)
    llm = LLM("bcg/tiny-qwen3", backend="hip", weights=ckpt, tensor_parallel_size=world, seed=5,
              max_model_len=1024, kv_cache_gb=0.5, max_batch_seqs=16)
    schemas = [P.honest_decision_schema(0, 50), P.vote_schema(P.BYZANTINE_VOTE_OPTIONS)]
    prompts = [f"<|im_start|>user\nagent_{i} proposes {i * 7}<|im_end|>\n<|im_start|>assistant\n" for i in range(6)]
    params = [SamplingParams(temperature=[0.0, 0.5][i % 2], max_tokens=40,
                             guided_decoding=GuidedDecodingParams(json=schemas[i % 2])) for i in range(6)]
    eng = llm.backend
    texts, raised = None, None
    if llm.is_driver:
        texts = [o.outputs[0].text for o in llm.generate(prompts, params)]
        eng.tp.custom.set_error()  # a peer "stalled": the next burst's barrier timed out
        try:
            llm.generate(prompts[:2], params[:2])
        except RuntimeError as exc:
            raised = str(exc)
    else:
        llm.serve_worker()
    calls = dict(eng.tp.custom.calls)
    captured = eng.graphs.captures if eng.graphs is not None else 0
    llm.shutdown()
    torch.cuda.synchronize()  # (the follower's last burst waits out the broken barrier: 3 s)
    torch.distributed.barrier()  # nobody unmaps its all-reduce buffers while a peer kernel may read them
    torch.save({"texts": texts, "raised": raised, "calls": calls, "captured": captured}, f"{out}.{rank}")
    groups.destroy()


def test_tp2_decode_graphs_match_eager_and_timeout_raises(tmp_path):
    from byzantine_consensus_llm_agents_amd.models.config import get_model_config
    from byzantine_consensus_llm_agents_amd.models.loader import save_hf_checkpoint
    from byzantine_consensus_llm_agents_amd.models.transformer import DecoderModel
    from byzantine_consensus_llm_agents_amd.ops import get_ops
    cfg = get_model_config("bcg/tiny-qwen3")
    ref = DecoderModel(cfg, get_ops("torch"), "cpu", torch.bfloat16)
    ref.init_random(seed=2, std=0.05)
    ckpt = str(tmp_path / "ckpt")
    save_hf_checkpoint(ref.hf_state_dict(), cfg, ckpt)
    res = {}
    for graphs in (True, False):
        out = str(tmp_path / f"g{int(graphs)}")
        mp.start_processes(_graph_worker, args=(2, _free_port(), ckpt, out, graphs), nprocs=2, join=True,
                           start_method="spawn")
        res[graphs] = [torch.load(f"{out}.{r}", weights_only=True) for r in range(2)]
    g0, e0 = res[True][0], res[False][0]
    assert g0["captured"] > 0 and e0["captured"] == 0
    assert g0["texts"] == e0["texts"]  # graph-captured TP decode == eager TP decode, token for token
    for t in g0["texts"]:
        json.loads(t)
    for r in (0, 1):
        assert res[True][r]["calls"].get(3, 0) > 0  # the fused all-reduce + RMSNorm kernel ran
    for graphs in (True, False):
        assert res[graphs][0]["raised"] and "all-reduce" in res[graphs][0]["raised"]
