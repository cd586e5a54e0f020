"""Headline benchmark: agent decisions/sec (node), 8 honest + 2 Byzantine BCG, Qwen3-14B bf16.

Metric (BASELINE.md "Measurement protocol"): accepted decide outputs +
accepted vote outputs per wall-clock second, summed over every GPU of the
node.  One "step" = one BCG round of every simulation running on the GPU (each
round: all agents' decide prompts in one engine call, all vote prompts in one
call, plus whatever retries the reference's retry ladder triggers).

Layout: one process per GPU (torchrun), data-parallel over independent
simulation seeds (``--sims-per-gpu`` games share each GPU's engine, which
serves them with continuous batching; a game that ends is replaced by a fresh
seed so the pool stays full).  With ``--tp > 1`` groups of GPUs form
tensor-parallel engines (RCCL all-reduce) fed by lock-step coalesced rounds.

Data: random-init weights of the real architecture and the synthetic
byte-level BPE tokenizer (no network for checkpoints); the budget-aware JSON
grammar guarantees schema-valid outputs from untrained weights, at the full
max_tokens (300 decide / 200 vote) -- a pessimistic decode length.

Timing: W warmup rounds, barrier + cuda.synchronize, K timed rounds,
barrier + synchronize; the max time over ranks; rank 0 prints one JSON line.
"""

import argparse
import json
import os
import random
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

BASELINE_VALUE = None  # the reference publishes no number


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3, help="timed BCG rounds")
    ap.add_argument("--warmup", type=int, default=1, help="untimed BCG rounds")
    ap.add_argument("--model", default="qwen3-14b")
    ap.add_argument("--honest", type=int, default=8)
    ap.add_argument("--byzantine", type=int, default=2)
    ap.add_argument("--sims-per-gpu", type=int, default=128)
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--max-rounds", type=int, default=50)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--backend", default="hip")
    ap.add_argument("--quantization", default=None, choices=["fp8"])
    ap.add_argument("--kv-cache-dtype", default="auto", choices=["auto", "fp8"],
                    help="fp8 halves KV bytes (reduced precision: never used for the bf16 headline)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--no-prefix-cache", action="store_true")
    ap.add_argument("--overlap-prefill", action="store_true",
                    help="prefill on a second HIP stream, concurrent with decode bursts (TP=1)")
    ap.add_argument("--no-custom-allreduce", action="store_true",
                    help="TP collectives through RCCL only (no xGMI one-/two-shot kernels)")
    ap.add_argument("--verbose", action="store_true")
    return ap.parse_args()


class SimPool:
    """S independent simulations, each on its own thread, sharing the engine.

    With continuous batching the simulations are NOT in lock-step: one game's
    retry phase overlaps another game's decide phase, keeping the decode batch
    full.  A game that ends is replaced by a fresh seed.  ``run(rounds)`` makes
    every simulation play exactly ``rounds`` rounds.
    """

    def __init__(self, n_sims, honest, byzantine, max_rounds, seed, rank):
        from byzantine_consensus_llm_agents_amd.bcg.simulation import BCGSimulation
        self.BCGSimulation = BCGSimulation
        self.honest, self.byzantine, self.max_rounds = honest, byzantine, max_rounds
        self.seed_base = seed * 100003 + rank * 7919
        self.next_seed = 0
        self.lock = threading.Lock()
        self.sims = [self._new_sim() for _ in range(n_sims)]
        self.games_finished = 0
        self.outcomes = {}

    def _new_sim(self):
        with self.lock:
            self.next_seed += 1
            seed = self.seed_base + self.next_seed
        return self.BCGSimulation(self.honest, self.byzantine, config={
            "max_rounds": self.max_rounds, "value_range": (0, 50), "consensus_threshold": 66.0,
            "verbose": False, "byzantine_awareness": "may_exist", "seed": seed})

    def run(self, rounds: int, llm=None, lockstep=False) -> int:
        """Every simulation plays `rounds` rounds; returns accepted decisions."""
        made = [0] * len(self.sims)
        errors = []

        def work(i):
            th = threading.current_thread()
            th._bcg_participant = lockstep
            th._bcg_order_key = (i,)
            try:
                for _ in range(rounds):
                    sim = self.sims[i]
                    before = sim.counters["decisions_accepted"] + sim.counters["votes_accepted"]
                    sim.run_round()
                    made[i] += sim.counters["decisions_accepted"] + sim.counters["votes_accepted"] - before
                    if sim.game.game_over:
                        o = sim.game.get_statistics().get("consensus_outcome")
                        with self.lock:
                            self.outcomes[o] = self.outcomes.get(o, 0) + 1
                            self.games_finished += 1
                        self.sims[i] = self._new_sim()
            except BaseException as exc:  # surface thread failures
                errors.append(exc)
            finally:
                if lockstep:
                    llm.unregister_client()

        if lockstep:
            for _ in self.sims:
                llm.register_client()
        threads = [threading.Thread(target=work, args=(i,)) for i in range(len(self.sims))]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        if errors:
            raise errors[0]
        return sum(made)


def _heartbeat(llm, stop: threading.Event, every: float = 30.0):
    """Progress line on stderr every `every` s (long runs must keep writing)."""
    t0 = time.perf_counter()
    while not stop.wait(every):
        st = dict(getattr(llm.backend, "stats", {}))
        print(f"[progress] {time.perf_counter() - t0:.0f}s {json.dumps(st)}", file=sys.stderr, flush=True)


def main():
    args = parse()
    # stdout carries exactly ONE line (the JSON result): anything else -- e.g. the
    # reference's console messages when an agent fails all JSON retries -- goes to stderr
    result_out, sys.stdout = sys.stdout, sys.stderr
    if os.environ.get("BCG_STACKS_AFTER"):  # debugging aid: dump every thread's stack periodically
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["BCG_STACKS_AFTER"]), repeat=True, file=sys.stderr)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.backend == "hip":
        torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl" if args.backend == "hip" else "gloo")

    from byzantine_consensus_llm_agents_amd.bcg import config as C
    from byzantine_consensus_llm_agents_amd.bcg.engine_agent import EngineAgent
    from byzantine_consensus_llm_agents_amd.engine.llm import LLM
    from byzantine_consensus_llm_agents_amd.models.config import ALIASES

    model = ALIASES.get(args.model, args.model)
    C.METRICS_CONFIG["save_results"] = False
    C.VLLM_CONFIG["model_name"] = model
    C.VLLM_CONFIG["tensor_parallel_size"] = args.tp
    C.VLLM_CONFIG["quantization"] = args.quantization
    C.ENGINE_CONFIG.update(backend=args.backend, budget_aware_json=True, seed=args.seed + rank // args.tp,
                           use_hip_graphs=not args.no_graphs, prefix_caching=not args.no_prefix_cache,
                           overlap_prefill=args.overlap_prefill, custom_allreduce=not args.no_custom_allreduce,
                           kv_cache_dtype=args.kv_cache_dtype)
    C.BCG_CONFIG["value_range"] = (0, 50)
    random.seed(args.seed + rank)

    t0 = time.perf_counter()
    llm = LLM(model, max_model_len=C.VLLM_CONFIG["max_model_len"],
              gpu_memory_utilization=C.VLLM_CONFIG["gpu_memory_utilization"],
              tensor_parallel_size=args.tp, backend=args.backend, seed=args.seed + rank // args.tp,
              quantization=args.quantization)
    # share the engine with every agent (same model name + config => no reload)
    EngineAgent._shared_llm = llm
    EngineAgent._shared_model_name = model
    EngineAgent._shared_model_config = dict(C.VLLM_CONFIG)
    init_s = time.perf_counter() - t0

    stop_hb = threading.Event()
    if rank == 0:
        threading.Thread(target=_heartbeat, args=(llm, stop_hb), daemon=True).start()
    lockstep = args.tp > 1  # TP ranks need identical batches: coalesced lock-step rounds
    if not lockstep:
        llm.start_continuous_batching()
    pool = SimPool(args.sims_per_gpu, args.honest, args.byzantine, args.max_rounds,
                   args.seed + rank // args.tp, rank // args.tp)
    if args.warmup:
        n = pool.run(args.warmup, llm, lockstep)
        if rank == 0:
            print(f"[warmup] {args.warmup} rounds/sim, decisions={n}", file=sys.stderr, flush=True)

    eng = getattr(llm.backend, "stats", {})
    stats0 = dict(eng)
    if world > 1:
        dist.barrier()
    if args.backend == "hip":
        torch.cuda.synchronize()
    t_start = time.perf_counter()
    decisions = pool.run(args.steps, llm, lockstep)
    if rank == 0:
        print(f"[timed] {args.steps} rounds/sim decisions={decisions} elapsed={time.perf_counter() - t_start:.2f}s",
              file=sys.stderr, flush=True)
    if args.backend == "hip":
        torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t_start

    # DP groups: only one rank per TP group contributes decisions
    mine = decisions if rank % args.tp == 0 else 0
    if world > 1:
        t = torch.tensor([mine, elapsed], dtype=torch.float64,
                         device="cuda" if args.backend == "hip" else "cpu")
        tot = t.clone()
        dist.all_reduce(tot[:1], op=dist.ReduceOp.SUM)
        mx = t[1:].clone()
        dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        total_decisions, elapsed = float(tot[0]), float(mx[0])
    else:
        total_decisions = float(mine)
    value = total_decisions / elapsed if elapsed > 0 else 0.0
    d_eng = {k: eng.get(k, 0) - stats0.get(k, 0) for k in eng}
    if rank == 0:
        line = {
            "metric": f"agent decisions/sec (node), {args.honest}h+{args.byzantine}b BCG {model.split('/')[-1]}; "
                      "consensus-rate parity",
            "value": round(value, 3), "unit": "decisions/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / max(args.steps, 1), 2),
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": (value / BASELINE_VALUE) if BASELINE_VALUE else None,
            "dtype": "fp8" if args.quantization == "fp8" else "bf16",
            "kv_cache_dtype": "fp8" if args.kv_cache_dtype == "fp8" else "bf16",
            "data": "synthetic (random-init weights, synthetic BPE tokenizer, budget-aware JSON grammar)",
            "config": {"model": model, "honest": args.honest, "byzantine": args.byzantine,
                       "global_batch": args.sims_per_gpu * (args.honest + args.byzantine) * (world // args.tp),
                       "sims_per_gpu": args.sims_per_gpu, "seq_len": C.VLLM_CONFIG["max_model_len"],
                       "max_tokens_decide": C.LLM_CONFIG["max_tokens_decide"],
                       "max_tokens_vote": C.LLM_CONFIG["max_tokens_vote"],
                       "parallelism": f"dp{world // args.tp}" + (f"xtp{args.tp}" if args.tp > 1 else ""),
                       "hip_graphs": not args.no_graphs, "prefix_caching": not args.no_prefix_cache,
                       "overlap_prefill": args.overlap_prefill,
                       "custom_allreduce": args.tp > 1 and not args.no_custom_allreduce},
            "detail": {"decisions": total_decisions, "elapsed_s": round(elapsed, 3), "init_s": round(init_s, 1),
                       "engine_per_rank": d_eng, "games_finished_rank0": pool.games_finished,
                       "outcomes_rank0": pool.outcomes,
                       "phases_rank0": llm.backend.timer.summary() if hasattr(llm.backend, "timer") else {}},
        }
        print(json.dumps(line), file=result_out, flush=True)
    stop_hb.set()
    llm.shutdown()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
