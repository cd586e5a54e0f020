"""Configuration registry for the Byzantine Consensus Game (BCG).

Same module-level dict schema as the reference (``bcg/config.py:7-77``): the
dicts are plain mutable objects and are mutated at runtime by the CLI
(``main.main``) and by ``run_simulation`` exactly like the reference does
(``bcg/main.py:1042``, ``:1097-1102``).  Everything specific to the MI355X
engine lives in ``ENGINE_CONFIG`` (new), so code written against the
reference's config keeps working unchanged.
"""

import os

# --- communication / network (reference bcg/config.py:7-15) -----------------
COMMUNICATION_CONFIG = {
    "protocol_type": "a2a_sim",
}

NETWORK_CONFIG = {
    "topology_type": "fully_connected",  # fully_connected | ring | grid | custom
    "custom_adjacency": None,
}

# --- model presets (reference bcg/config.py:20-25) + the plumbing model ------
MODEL_PRESETS = {
    "qwen3-8b": "Qwen/Qwen3-8B",
    "qwen3-14b": "Qwen/Qwen3-14B",
    "qwen3-32b": "Qwen/Qwen3-32B",
    "mistral-22b": "mistralai/Mistral-Small-Instruct-2409",
    "qwen2.5-0.5b": "Qwen/Qwen2.5-0.5B-Instruct",
}

ACTIVE_MODEL = "qwen3-14b"

# Engine knobs keep the reference's key names (bcg/config.py:33-41).  On the
# MI355X engine `max_num_seqs` is only honoured in reference-emulation mode
# (ENGINE_CONFIG["honor_max_num_seqs"]); `quantization` selects the fp8 path.
VLLM_CONFIG = {
    "model_name": MODEL_PRESETS[ACTIVE_MODEL],
    "max_model_len": 8192,
    "gpu_memory_utilization": 0.9,
    "tensor_parallel_size": 1,
    "max_num_seqs": 4,
    "quantization": None,
    "disable_qwen3_thinking": True,
}

AGENT_CONFIG = {
    "use_structured_output": True,
    "use_batched_inference": True,
}

# Single source of truth for sampling (reference bcg/config.py:52-58).
LLM_CONFIG = {
    "temperature_decide": 0.5,
    "temperature_vote": 0.3,
    "max_tokens_decide": 300,
    "max_tokens_vote": 200,
    "max_json_retries": 3,
}

BCG_CONFIG = {
    "num_honest": 8,
    "num_byzantine": 0,
    "value_range": (0, 50),
    "consensus_threshold": 66.0,
    "max_rounds": 50,
}

METRICS_CONFIG = {
    "track_convergence": True,
    "track_byzantine_impact": True,
    "track_communication": True,
    "save_results": True,
    "generate_plots": False,
    "results_dir": "results",
}

# --- MI355X engine (new) -----------------------------------------------------
# backend: "hip"  -> in-process MI355X engine (HIP kernels, RCCL for TP)
#          "torch"-> same engine on torch reference ops (CPU / debugging)
#          "fake" -> scripted schema-valid responses, no model (plumbing/tests)
ENGINE_CONFIG = {
    "backend": os.environ.get("BCG_ENGINE", "auto"),
    "weights": os.environ.get("BCG_WEIGHTS", "auto"),  # auto | random | <dir with safetensors>
    "dtype": os.environ.get("BCG_DTYPE", "bfloat16"),  # activation/weight dtype (float32: CPU parity tests)
    "kv_block_size": 16,
    "seed": None,                  # None = unseeded (reference behaviour)
    "budget_aware_json": False,    # force closing JSON before max_tokens
    # benchmark grammar for untrained weights: every property emitted, free-text fields with at
    # least this many visible characters (the simulator's validity rules then hold, as for a
    # trained model's outputs); 0 = the reference's schemas as given
    "validity_aware_json": 0,
    "ascii_text_json": False,
    "max_whitespace": 4,           # JSON grammar: max consecutive whitespace chars
    "prefix_caching": True,
    "use_hip_graphs": True,
    "max_batch_seqs": 768,
    "prefill_chunk_tokens": 16384,
    "honor_max_num_seqs": False,
    "kv_cache_gb": None,           # None = size from gpu_memory_utilization
    "kv_cache_dtype": os.environ.get("BCG_KV_CACHE_DTYPE", "auto"),  # auto (bf16) | fp8 (e4m3fn)
    # decode bursts a prompt may wait so prefill runs in full chunks (0 = admit immediately);
    # only while >= admit_min_live rows decode.  3 vs 0, two A/B pairs on one GPU: 31.0k / 31.5k
    # vs 30.6k / 30.8k tokens/s (profiles/bench_r2_ab*_a*.json)
    "admit_max_wait": int(os.environ.get("BCG_ADMIT_MAX_WAIT", "3")),
    # decode steps per burst (graph replays between two host polls of the completion state); a
    # finished row idles until the poll after the burst that follows its last step
    "poll_every": int(os.environ.get("BCG_POLL_EVERY", "8")),
    # run only full prefill chunks while the decode batch is fed: a wave's partial last chunk
    # waits (its prompts pending with their KV so far) up to this many more bursts for the
    # next wave (engine.py `_hold_tail`); 0 = run it at once.  2 vs 0, two A/B pairs in opposite
    # order on one GPU: 38.4k / 38.3k vs 38.0k / 37.9k tokens/s (no ragged tail chunks;
    # profiles/r6_carry_ab)
    "prefill_carry_bursts": int(os.environ.get("BCG_PREFILL_CARRY", "2")),
    # tests only: run the model with this many decoder layers (real layer shapes, reduced depth)
    "num_layers_override": None,
}
