"""Data-parallel experiment sweep: many independent games (seeds) over every GPU of a node.

The reference's experiments were cluster sweeps of independent runs driven
through ``run_simulation`` (``bcg/main.py:1073-1141``; the driver itself is
not in the repo, SURVEY.md §2.2 "DP over seeds", §7.2 step 6).  Here one
launch covers the whole sweep:

* one process per GPU (``torchrun``), TP groups of ``--tp`` consecutive ranks
  (RCCL + xGMI all-reduce), DP replicas over the groups;
* replicas pull seeds one at a time from a node-wide counter (TCPStore), so
  uneven game lengths never leave a replica idle while another still holds a
  static share; each replica plays ``--concurrency`` games at a time on ONE
  engine -- their decide/vote batches share the continuously-batched decode
  (TP groups: the group's rank 0 drives, the followers replay its schedule);
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


class SeedQueue:
    """Seeds handed out one at a time; shared by every DP replica of the node.

    Replicas pull the next seed index from an atomic counter in the process
    group's TCPStore (``store.add``), so a replica that drew short games takes
    more of them -- no replica idles at the tail while another still has a
    static share to play.  Single process: a local counter.
    """

    def __init__(self, seeds: List[int], store=None, key: str = "bcg_sweep_next"):
        self.seeds, self.store, self.key = list(seeds), store, key
        self._lock = threading.Lock()
        self._next = 0

    def pop(self):
        if self.store is not None:
            i = int(self.store.add(self.key, 1)) - 1
        else:
            with self._lock:
                i, self._next = self._next, self._next + 1
        return self.seeds[i] if i < len(self.seeds) else None


def run_games(seeds, args, llm=None, checkpoint=None) -> List[Dict]:
    """Play seeds with up to `args.concurrency` games in flight (worker threads).

    `seeds`: a list (played by this process alone) or a :class:`SeedQueue`
    shared with the other replicas.  `checkpoint`: optional open text file;
    each finished game is appended as one JSON line.
    """
    lo, hi = map(int, args.value_range.split("-"))
    q = seeds if isinstance(seeds, SeedQueue) else SeedQueue(seeds)
    results, errors = [], []
    ck_lock = threading.Lock()
    n_workers = max(1, min(args.concurrency, len(q.seeds)))

    def worker(i):
        threading.current_thread()._bcg_order_key = (i,)
        try:
            while True:
                seed = q.pop()
                if seed is None:
                    return
                rec = play_game(seed, args.honest, args.byzantine, args.rounds, (lo, hi),
                                args.byzantine_awareness)
                rec["finished_at"] = time.perf_counter()
                results.append(rec)
                if checkpoint is not None:
                    with ck_lock:
                        checkpoint.write(json.dumps({k: v for k, v in rec.items() if k != "finished_at"}) + "\n")
                        checkpoint.flush()
        except BaseException as exc:
            errors.append(exc)

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
    from ..utils.threads import rank_thread_budget
    rank_thread_budget(int(os.environ.get("WORLD_SIZE", "1")))  # before torch / tokenizer pools start
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
    from .prompts import all_schemas
    llm.precompile(all_schemas(lo, hi))  # every rank, same order (TP: identical FSM row bases)

    ctrl = None
    if lay.world > 1:
        import torch.distributed as dist
        # results / barriers on a CPU group: never queued behind the engine's HIP work
        ctrl = dist.new_group(backend="gloo") if dist.get_backend() != "gloo" else None
    done = load_checkpoints(args.out) if args.resume else {}
    if lay.world > 1:  # every rank has read the checkpoints before anyone appends
        dist.barrier(group=ctrl)
    all_seeds = [args.seed0 + i for i in range(args.seeds)]
    todo = [s for s in all_seeds if s not in done]
    store = None
    if lay.world > 1:
        from torch.distributed.distributed_c10d import _get_default_store
        store = _get_default_store()
    queue_ = SeedQueue(todo, store, key=f"bcg_sweep_next_{args.seed0}_{len(todo)}")
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
    games = []
    try:
        if llm.is_driver:  # the group's rank 0 plays; TP followers replay its schedule
            llm.start_continuous_batching()
            games = run_games(queue_, args, llm, checkpoint=ck)
        else:
            llm.serve_worker()
    finally:
        if ck is not None:
            ck.close()
        if llm.is_driver:
            llm.shutdown()  # releases the followers
    elapsed = time.perf_counter() - t0
    busy = max((g["finished_at"] for g in games), default=t0 + elapsed) - t0
    for g in games:
        g.pop("finished_at", None)

    if lay.world > 1:
        gathered = [None] * lay.world
        dist.all_gather_object(gathered, {"games": games, "elapsed": elapsed, "busy": busy,
                                          "driver": llm.is_driver}, group=ctrl)
        games = sorted((g for part in gathered for g in part["games"]), key=lambda r: r["seed"])
        elapsed = max(part["elapsed"] for part in gathered)
        drivers = [p for p in gathered if p["driver"]]
        # idle tail: how long replicas waited for the slowest one after their last game
        tail = [elapsed - p["busy"] for p in drivers]
    else:
        tail = [elapsed - busy]
    if done:
        resumed = [done[s] for s in all_seeds if s in done]
        games = sorted(games + resumed, key=lambda r: r["seed"])
    summary = summarize(games, elapsed, lay.world)
    summary["resumed_games"] = len(done)
    summary["replica_idle_tail_frac"] = round(max(tail) / elapsed, 4) if elapsed > 0 else 0.0
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
    if not llm.is_driver:
        llm.shutdown()
    EngineAgent._shared_llm = None
    destroy()
    return summary


if __name__ == "__main__":
    main()
