"""Data-parallel experiment sweep: many independent games (seeds) over every GPU of a node.

The reference's experiments were cluster sweeps of independent runs driven
through ``run_simulation`` (``bcg/main.py:1073-1141``; the driver itself is
not in the repo, SURVEY.md §2.2 "DP over seeds", §7.2 step 6).  Here one
launch covers the whole sweep:

* one process per GPU (``torchrun``), TP groups of ``--tp`` consecutive ranks
  (RCCL + xGMI all-reduce), DP replicas over the groups;
* every replica plays its share of the seeds (round-robin), ``--concurrency``
  games at a time on ONE engine -- their decide/vote batches share the
  continuously-batched decode (TP groups: coalesced lock-step batches);
* each game is exactly the reference's ``run_simulation`` loop (round until
  ``game.game_over``) with a seeded ``ByzantineConsensusGame``;
* rank 0 gathers every game's ``get_statistics()`` and writes one JSON: the
  consensus-outcome distribution (valid / invalid / none / timeout -- the
  BASELINE.md quality-parity metric), mean rounds / quality score, and
  decisions per second over the node;
* checkpoint / resume (the reference has neither): every
  finished game is appended to ``<out>.rank<R>.jsonl`` as it completes;
  ``--resume`` reloads all those records and only plays the missing seeds.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m byzantine_consensus_llm_agents_amd.bcg.sweep --seeds 64 --honest 8 --byzantine 2
"""

import argparse
import json
import os
import queue
import random
import sys
import threading
import time
from typing import Dict, List

OUTCOMES = ("valid", "invalid", "none", "timeout")

PER_GAME_KEYS = ("consensus_outcome", "total_rounds", "consensus_reached", "consensus_value",
                 "consensus_quality_score", "termination_reason", "honest_agents_won", "convergence_speed")


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="BCG seed sweep (data-parallel over GPUs)")
    p.add_argument("--seeds", type=int, default=8, help="number of games")
    p.add_argument("--seed0", type=int, default=0, help="first game seed")
    p.add_argument("--honest", type=int, default=8)
    p.add_argument("--byzantine", type=int, default=2)
    p.add_argument("--rounds", type=int, default=50, help="max rounds per game")
    p.add_argument("--value-range", type=str, default="0-50")
    p.add_argument("--byzantine-awareness", default="may_exist", choices=["may_exist", "none_exist"])
    p.add_argument("--model", default=None, help="preset key or HF name (default: config ACTIVE_MODEL)")
    p.add_argument("--tp", type=int, default=1)
    p.add_argument("--engine", default=None, choices=["auto", "hip", "torch", "fake"])
    p.add_argument("--weights", default=None)
    p.add_argument("--quantization", default=None, choices=["fp8"])
    p.add_argument("--concurrency", type=int, default=64, help="games in flight per engine")
    p.add_argument("--budget-aware-json", action="store_true")
    p.add_argument("--engine-seed", type=int, default=None, help="sampler seed (default: seed0)")
    p.add_argument("--out", default=os.path.join("results", "sweep.json"))
    p.add_argument("--resume", action="store_true", help="skip seeds already checkpointed next to --out")
    return p


def checkpoint_path(out: str, rank: int) -> str:
    return f"{out}.rank{rank}.jsonl"


def load_checkpoints(out: str) -> Dict[int, Dict]:
    """Every game record checkpointed by any rank of an earlier (possibly killed) run."""
    import glob
    done = {}
    for path in sorted(glob.glob(glob.escape(out) + ".rank*.jsonl")):
        with open(path) as fh:
            for line in fh:
                line = line.strip()
                if not line:
                    continue
                try:
                    rec = json.loads(line)
                except json.JSONDecodeError:  # torn last line of a killed run
                    continue
                done[rec["seed"]] = rec
    return done


def play_game(seed: int, honest: int, byzantine: int, max_rounds: int, value_range, awareness: str) -> Dict:
    """One complete game (reference run_simulation semantics) -> per-game record."""
    from .simulation import BCGSimulation
    sim = BCGSimulation(honest, byzantine, config={
        "max_rounds": max_rounds, "value_range": tuple(value_range), "consensus_threshold": 66.0,
        "verbose": False, "byzantine_awareness": awareness, "seed": seed})
    while not sim.game.game_over:
        sim.run_round()
    stats = sim.game.get_statistics()
    rec = {k: stats.get(k) for k in PER_GAME_KEYS}
    rec["seed"] = seed
    rec["decisions"] = sim.counters["decisions_accepted"] + sim.counters["votes_accepted"]
    return rec


def run_games(seeds: List[int], args, llm=None, lockstep: bool = False, checkpoint=None) -> List[Dict]:
    """Play `seeds` with up to `args.concurrency` games in flight (worker threads).

    `checkpoint`: optional open text file; each finished game is appended as one JSON line.
    """
    lo, hi = map(int, args.value_range.split("-"))
    work: "queue.Queue[int]" = queue.Queue()
    for s in seeds:
        work.put(s)
    results, errors = [], []
    ck_lock = threading.Lock()
    n_workers = max(1, min(args.concurrency, len(seeds)))

    def worker(i):
        th = threading.current_thread()
        th._bcg_participant = lockstep
        th._bcg_order_key = (i,)
        try:
            while True:
                try:
                    seed = work.get_nowait()
                except queue.Empty:
                    return
                rec = play_game(seed, args.honest, args.byzantine, args.rounds, (lo, hi),
                                args.byzantine_awareness)
                results.append(rec)
                if checkpoint is not None:
                    with ck_lock:
                        checkpoint.write(json.dumps(rec) + "\n")
                        checkpoint.flush()
        except BaseException as exc:
            errors.append(exc)
        finally:
            if lockstep:
                llm.unregister_client()

    if lockstep:
        # TP ranks of a group play the same seeds in the same worker slots: the
        # coalescer turns their calls into identical batches on every rank
        for _ in range(n_workers):
            llm.register_client()
    threads = [threading.Thread(target=worker, args=(i,)) for i in range(n_workers)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errors:
        raise errors[0]
    return sorted(results, key=lambda r: r["seed"])


def summarize(games: List[Dict], elapsed: float, n_gpus: int) -> Dict:
    n = len(games)
    counts = {o: sum(1 for g in games if g["consensus_outcome"] == o) for o in OUTCOMES}
    decisions = sum(g["decisions"] for g in games)

    def mean(key):
        vals = [g[key] for g in games if isinstance(g.get(key), (int, float))]
        return round(sum(vals) / len(vals), 4) if vals else None

    return {"games": n, "outcomes": counts,
            "outcome_rates": {o: round(c / n, 4) if n else 0.0 for o, c in counts.items()},
            "consensus_rate": round(counts["valid"] / n, 4) if n else 0.0,
            "mean_rounds": mean("total_rounds"), "mean_quality_score": mean("consensus_quality_score"),
            "decisions": decisions, "elapsed_s": round(elapsed, 3), "n_gpus": n_gpus,
            "decisions_per_s": round(decisions / elapsed, 3) if elapsed > 0 else None}


def main(argv=None) -> Dict:
    args = build_parser().parse_args(argv)
    saved_stdout, sys.stdout = sys.stdout, sys.stderr  # agents' console messages; the summary line stays alone
    try:
        return _main(args)
    finally:
        sys.stdout = saved_stdout


def _main(args) -> Dict:
    from ..parallel.groups import destroy, env_layout, init_distributed
    from . import config as C
    from .engine_agent import EngineAgent

    lay = init_distributed()
    lay = env_layout(args.tp) if lay.world > 1 else lay
    if lay.world % args.tp:
        raise SystemExit(f"world {lay.world} not divisible by --tp {args.tp}")
    dp, dp_rank = lay.world // args.tp, lay.rank // args.tp

    C.METRICS_CONFIG["save_results"] = False
    lo, hi = map(int, args.value_range.split("-"))
    C.BCG_CONFIG["value_range"] = (lo, hi)
    if args.model:
        C.VLLM_CONFIG["model_name"] = C.MODEL_PRESETS.get(args.model, args.model)
    C.VLLM_CONFIG["tensor_parallel_size"] = args.tp
    if args.quantization:
        C.VLLM_CONFIG["quantization"] = args.quantization
    if args.engine:
        C.ENGINE_CONFIG["backend"] = args.engine
    if args.weights:
        C.ENGINE_CONFIG["weights"] = args.weights
    if args.budget_aware_json:
        C.ENGINE_CONFIG["budget_aware_json"] = True
    engine_seed = args.seed0 if args.engine_seed is None else args.engine_seed
    from ..engine.llm import LLM, resolve_backend
    if resolve_backend(args.engine) != "fake":
        # decorrelate the replicas' sampling streams (TP ranks share rank 0's: the engine
        # broadcasts it); the scripted backend is a pure function of (prompt, schema,
        # seed), so there a game's transcript depends on its game seed alone
        engine_seed += dp_rank
    C.ENGINE_CONFIG["seed"] = engine_seed
    random.seed(args.seed0 + dp_rank)

    model = C.VLLM_CONFIG["model_name"]
    llm = LLM(model, max_model_len=C.VLLM_CONFIG["max_model_len"],
              gpu_memory_utilization=C.VLLM_CONFIG["gpu_memory_utilization"], tensor_parallel_size=args.tp,
              quantization=C.VLLM_CONFIG.get("quantization"), seed=engine_seed)
    EngineAgent._shared_llm, EngineAgent._shared_model_name = llm, model
    EngineAgent._shared_model_config = dict(C.VLLM_CONFIG)
    lockstep = args.tp > 1
    if not lockstep:
        llm.start_continuous_batching()

    done = load_checkpoints(args.out) if args.resume else {}
    if lay.world > 1:  # every rank has read the checkpoints before anyone appends
        import torch.distributed as dist
        dist.barrier()
    all_seeds = [args.seed0 + i for i in range(args.seeds)]
    todo = [s for s in all_seeds if s not in done]
    seeds = [s for i, s in enumerate(todo) if i % dp == dp_rank]  # identical split on every rank
    ck = None
    if lay.tp_rank == 0:
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        path = checkpoint_path(args.out, lay.rank)
        torn = args.resume and os.path.exists(path) and os.path.getsize(path) > 0 and \
            open(path, "rb").read()[-1:] != b"\n"
        ck = open(path, "a" if args.resume else "w")
        if torn:
            ck.write("\n")  # seal a torn last line so the next record parses
    t0 = time.perf_counter()
    try:
        games = run_games(seeds, args, llm, lockstep, checkpoint=ck)
    finally:
        if ck is not None:
            ck.close()
    elapsed = time.perf_counter() - t0
    mine = games if lay.tp_rank == 0 else []

    if lay.world > 1:
        import torch.distributed as dist
        gathered = [None] * lay.world
        dist.all_gather_object(gathered, {"games": mine, "elapsed": elapsed})
        games = sorted((g for part in gathered for g in part["games"]), key=lambda r: r["seed"])
        elapsed = max(part["elapsed"] for part in gathered)
    if done:
        resumed = [done[s] for s in all_seeds if s in done]
        games = sorted(games + resumed, key=lambda r: r["seed"])
    summary = summarize(games, elapsed, lay.world)
    summary["resumed_games"] = len(done)
    summary["config"] = {"model": model, "honest": args.honest, "byzantine": args.byzantine,
                         "max_rounds": args.rounds, "value_range": [lo, hi], "tp": args.tp, "dp": dp,
                         "byzantine_awareness": args.byzantine_awareness, "seed0": args.seed0,
                         "backend": llm.backend_name, "quantization": args.quantization}
    summary["per_game"] = games
    if lay.rank == 0:
        os.makedirs(os.path.dirname(os.path.abspath(args.out)), exist_ok=True)
        with open(args.out, "w") as fh:
            json.dump(summary, fh, indent=2)
        brief = {k: v for k, v in summary.items() if k != "per_game"}
        print(json.dumps(brief), file=sys.__stdout__ if sys.stdout is sys.stderr else sys.stdout, flush=True)
    llm.shutdown()
    EngineAgent._shared_llm = None
    destroy()
    return summary


if __name__ == "__main__":
    main()
