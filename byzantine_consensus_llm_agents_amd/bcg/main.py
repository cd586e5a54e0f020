"""Command line entry point and batch-experiment API.

Parity target: reference ``bcg/main.py`` ``main`` (:998-1070) and
``run_simulation`` (:1073-1141).  The reference flags are unchanged
(``--honest --byzantine --rounds --threshold --value-range
--byzantine-awareness --verbose``) and mutate the config dicts the same way.
New optional flags (``--model``, ``--tp``, ``--seed``, ``--engine``,
``--weights``, ``--budget-aware-json``) only touch ``VLLM_CONFIG`` /
``ENGINE_CONFIG`` when given.
"""

import argparse
import os

from .config import (AGENT_CONFIG, BCG_CONFIG, ENGINE_CONFIG, METRICS_CONFIG, MODEL_PRESETS,
                     VLLM_CONFIG)
from .engine_agent import EngineAgent
from .simulation import BCGSimulation


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Byzantine Consensus Game Simulation")
    p.add_argument("--honest", type=int, default=None, help="Number of honest agents (default: from config)")
    p.add_argument("--byzantine", type=int, default=None,
                   help="Number of Byzantine agents (default: from config, can be 0)")
    p.add_argument("--rounds", type=int, default=None, help="Max number of rounds (default: from config)")
    p.add_argument("--threshold", type=float, default=None,
                   help="Majority agreement percentage required (default: 66 percent)")
    p.add_argument("--value-range", type=str, default=None, help="Value range as 'min-max' (default: 0-50)")
    p.add_argument("--byzantine-awareness", type=str, default="may_exist",
                   choices=["may_exist", "none_exist"],
                   help="Whether honest agents are told Byzantine agents may exist (default: may_exist)")
    p.add_argument("--verbose", action="store_true",
                   help="Print detailed output to terminal (default: minimal for cluster)")
    # MI355X engine extensions (all optional)
    p.add_argument("--model", type=str, default=None,
                   help="Model preset key or HF name (default: config ACTIVE_MODEL)")
    p.add_argument("--tp", type=int, default=None, help="Tensor-parallel degree")
    p.add_argument("--seed", type=int, default=None, help="Seed the game and sampler (default: unseeded)")
    p.add_argument("--engine", type=str, default=None, choices=["auto", "hip", "torch", "fake"])
    p.add_argument("--weights", type=str, default=None, help="'random' or a safetensors directory")
    p.add_argument("--quantization", type=str, default=None, choices=["fp8"],
                   help="fp8 (e4m3fn) projection GEMMs (the reference only logs this key)")
    p.add_argument("--kv-cache-dtype", type=str, default=None, choices=["auto", "fp8"],
                   help="KV cache element type: auto (= bf16) or fp8 (e4m3fn, half the bytes)")
    p.add_argument("--budget-aware-json", action="store_true",
                   help="Close the JSON before max_tokens instead of truncating")
    return p


def _apply_engine_flags(args):
    if args.model:
        VLLM_CONFIG["model_name"] = MODEL_PRESETS.get(args.model, args.model)
    if args.tp:
        VLLM_CONFIG["tensor_parallel_size"] = args.tp
    if args.engine:
        ENGINE_CONFIG["backend"] = args.engine
    if args.weights:
        ENGINE_CONFIG["weights"] = args.weights
    if args.quantization:
        VLLM_CONFIG["quantization"] = args.quantization
    if args.seed is not None:
        ENGINE_CONFIG["seed"] = args.seed
    if args.budget_aware_json:
        ENGINE_CONFIG["budget_aware_json"] = True
    if args.kv_cache_dtype:
        ENGINE_CONFIG["kv_cache_dtype"] = args.kv_cache_dtype


def main(argv=None):
    args = build_parser().parse_args(argv)
    num_honest = args.honest if args.honest is not None else BCG_CONFIG["num_honest"]
    num_byzantine = args.byzantine if args.byzantine is not None else BCG_CONFIG["num_byzantine"]
    max_rounds = args.rounds if args.rounds is not None else BCG_CONFIG["max_rounds"]
    threshold = args.threshold if args.threshold is not None else BCG_CONFIG["consensus_threshold"]
    if args.value_range:
        try:
            lo, hi = map(int, args.value_range.split("-"))  # negatives unsupported, as in the reference
        except ValueError:
            print(f"Error: Invalid value range format '{args.value_range}'. Use 'min-max' (e.g., 0-50)")
            return
        value_range = (lo, hi)
    else:
        value_range = BCG_CONFIG["value_range"]

    config = {"max_rounds": max_rounds, "consensus_threshold": threshold, "value_range": value_range,
              "verbose": args.verbose, "byzantine_awareness": args.byzantine_awareness}
    if args.seed is not None:
        config["seed"] = args.seed
    BCG_CONFIG["value_range"] = value_range
    AGENT_CONFIG["verbose"] = args.verbose
    _apply_engine_flags(args)

    bar = "=" * 60
    print(f"\n{bar}")
    print("Configuration:")
    print(f"  Honest agents: {num_honest}")
    print(f"  Byzantine agents: {num_byzantine}")
    print(f"  Value range: {value_range[0]}-{value_range[1]}")
    print(f"  Max rounds: {max_rounds}")
    print(f"  Consensus threshold: {threshold}%")
    print(f"  Byzantine awareness: {args.byzantine_awareness}")
    print(f"{bar}\n")

    sim = BCGSimulation(num_honest=num_honest, num_byzantine=num_byzantine, config=config)
    try:
        sim.run()
    finally:
        EngineAgent.shutdown()


def run_simulation(n_agents: int = 8, max_rounds: int = 50, model_name: str = None,
                   byzantine_count: int = 0, byzantine_awareness: str = "may_exist",
                   seed=None) -> dict:
    """One simulation without file output; returns ``{"metrics": stats}``."""
    saved = (METRICS_CONFIG["save_results"], METRICS_CONFIG.get("generate_plots", True))
    METRICS_CONFIG["save_results"] = False
    METRICS_CONFIG["generate_plots"] = False
    if model_name:
        VLLM_CONFIG["model_name"] = model_name
    config = {
        "max_rounds": max_rounds,
        "consensus_threshold": BCG_CONFIG.get("consensus_threshold", 66.0),
        "value_range": BCG_CONFIG.get("value_range", (0, 50)),
        "verbose": os.environ.get("VERBOSE", "0") == "1",
        "byzantine_awareness": byzantine_awareness,
    }
    if seed is not None:
        config["seed"] = seed
    try:
        sim = BCGSimulation(num_honest=n_agents - byzantine_count, num_byzantine=byzantine_count,
                            config=config)
        while not sim.game.game_over:
            sim.run_round()
        stats = sim.game.get_statistics()
        stats["byzantine_awareness"] = byzantine_awareness
        return {"metrics": stats}
    finally:
        METRICS_CONFIG["save_results"], METRICS_CONFIG["generate_plots"] = saved


if __name__ == "__main__":
    main()
