"""Headline benchmark: agent decisions/sec (node), 8 honest + 2 Byzantine BCG, Qwen3-14B bf16.

Metric (BASELINE.md "Measurement protocol"): accepted decide outputs +
accepted vote outputs per wall-clock second, summed over every GPU of the
node.  Retries cost time but are not counted.

Unit of work.  ``--sims-per-gpu`` independent games (seeds) run continuously
on each engine, each on its own thread; a game that ends is replaced by a
fresh seed, so the continuously-batched decode stays full (steady state).  One
"step" is one fixed wall-clock window of ``--window-s`` seconds of that pool;
its decisions are the accepted decide/vote outputs completed inside it.

Steady state of WHOLE games ("wall-clock covers full simulations"): a
fresh pool would put every game in its first rounds at once (short prompts), so
each slot's first game is first burned in for A ~ Geometric(``--age-p``) rounds on
a scripted CPU engine (``SimPool.burn_in``: the age law of a long-running pool),
the pool then runs until every slot has finished a decide phase (``--fill-max-s``;
the start-up prefill wave is over) -- this fill counts toward the W warmup windows
(full batch, warm prefix cache, every decode graph captured) -- and K windows are
timed between a barrier +
``torch.cuda.synchronize()`` on both sides; the elapsed time is the max over
ranks and the decision count the sum over DP replicas.  Nothing is skipped
inside the timed region: every decision counted was fully generated,
FSM-guided, parsed and validated by the game.

Layout: one process per GPU.  ``--gpus N`` with no ``WORLD_SIZE`` in the
environment launches N ranks itself (a ``torch.distributed.run`` child
process, started before this process touches the GPU).  DP over seeds across
engines; ``--tp > 1`` groups consecutive ranks into one tensor-parallel engine
(rank 0 of the group schedules, the others execute its plans).

Data: random-init weights of the real architecture and the synthetic
byte-level BPE tokenizer (no network for checkpoints); the budget-aware JSON
grammar guarantees schema-valid outputs from untrained weights at the full
max_tokens (300 decide / 200 vote) -- a pessimistic decode length -- and its
validity-aware form (every property emitted, >= 10 visible characters per
free-text field) makes them pass the simulator's validity rules, as a trained
model's outputs do; ``--plain-grammar`` drops that (a random model then sends
~30 % of its outputs down the retry ladder: ``detail.retry``).  Free text is
printable ASCII (``--unicode-text`` lifts that): a random model's escapes and
multi-byte characters re-tokenise at several tokens per character once later
prompts quote them, and late-game prompts then hit the context limit, far
outside the reference's bounded prompt sizes.  ``detail.prompt_tokens``
(p50/p95/max per phase) and ``detail.context`` (prompts rejected or cut at the
context limit) report the envelope the timed region actually saw.

Deadline guard: if the run would pass ``--deadline-s`` (from process start),
the timed loop stops early and the JSON line reports the windows actually
timed (``steps``) -- the result line is always printed.
"""

import argparse
import json
import os
import random
import socket
import subprocess
import sys
import threading
import time

T_PROCESS0 = time.perf_counter()
ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

BASELINE_VALUE = None  # the reference publishes no number
# the bench grammar's visible-character floor of free-text fields (engine validity_aware_json):
# the simulator's validity rules (strategy >= 3, reasoning >= 10 stripped chars) then hold for
# the random model's outputs, as they do for a trained model's
VALIDITY_MIN_VISIBLE = 10


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20, help="timed windows")
    ap.add_argument("--warmup", type=int, default=5, help="untimed warmup windows")
    ap.add_argument("--window-s", type=float, default=12.0,
                    help="seconds per step (window); 12 s x 20 steps = 240 s timed (VERDICT r3: resolvable headline)")
    ap.add_argument("--deadline-s", type=float, default=540.0,
                    help="stop timing early rather than run past this many seconds from process start")
    ap.add_argument("--model", default="qwen3-14b")
    ap.add_argument("--honest", type=int, default=8)
    ap.add_argument("--byzantine", type=int, default=2)
    ap.add_argument("--sims-per-gpu", type=int, default=128)
    ap.add_argument("--max-batch-seqs", type=int, default=None,
                    help="decode batch cap (rows); default ENGINE_CONFIG['max_batch_seqs']")
    ap.add_argument("--ramp-s", type=float, default=None,
                    help="start the games spread over this many seconds (default: half the warmup)")
    ap.add_argument("--age-p", type=float, default=0.15,
                    help="age-diverse pool: each slot's first game is burned in for A ~ Geometric(p) rounds "
                         "(scripted CPU engine, before any timed window); 0 = every game starts fresh")
    ap.add_argument("--burnin-chars", default="320,420",
                    help="internal_strategy,public_reasoning characters of the burn-in outputs "
                         "(measured means of the engine's outputs: detail.age_mix.output_chars)")
    ap.add_argument("--fill-max-s", type=float, default=280.0,
                    help="wait (at most this long) until every game has finished its first decide "
                         "phase: the start-up prefill wave is over; the fill counts toward the warmup windows")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--max-rounds", type=int, default=50)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--backend", default="hip")
    ap.add_argument("--quantization", default=None, choices=["fp8"])
    ap.add_argument("--kv-cache-dtype", default="auto", choices=["auto", "fp8"],
                    help="fp8 halves KV bytes (reduced precision: never used for the bf16 headline)")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--no-prefix-cache", action="store_true")
    ap.add_argument("--plain-grammar", action="store_true",
                    help="the reference's schemas as given (no validity-aware bench grammar): a random model "
                         "then closes strings early / skips optional fields and ~30 %% of its outputs retry")
    ap.add_argument("--unicode-text", action="store_true",
                    help="free text may hold escapes and multi-byte UTF-8 (default: printable ASCII, as an "
                         "English-speaking trained model writes; a random model's unicode re-tokenises at "
                         "several tokens per character and late-game prompts reach the context limit)")
    ap.add_argument("--no-custom-allreduce", action="store_true",
                    help="TP collectives through RCCL only (no xGMI one-/two-shot kernels)")
    ap.add_argument("--kv-cache-gb", type=float, default=None,
                    help="KV cache size per engine (default: from free memory x gpu_memory_utilization)")
    ap.add_argument("--one-device", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank on cuda:0, gloo process group, the xGMI "
                         "all-reduce kernels forced over IPC peer buffers (never for measurements)")
    ap.add_argument("--verbose", action="store_true")
    return ap.parse_args(argv)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(args) -> int:
    """`--gpus N` without a launcher: run N ranks as a torchrun CHILD process.

    Nothing here touches the GPU (no HIP call before the ranks exist); the
    parent only waits and returns the child's exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", BCG_BENCH_T0=repr(time.time() - (time.perf_counter() - T_PROCESS0)))
    return subprocess.call(cmd, env=env)  # (each rank sets its own thread budget: rank_thread_budget)


class SimPool:
    """S independent games on their own threads, sharing one engine, running until stopped.

    The seed of the game slot ``i`` plays after ``g`` finished games is a pure
    function of (seed, replica, i, g), so the game sequence is reproducible and
    identical on every rank that derives it.
    """

    def __init__(self, n_sims, honest, byzantine, max_rounds, seed, replica):
        from byzantine_consensus_llm_agents_amd.bcg.simulation import BCGSimulation
        self.BCGSimulation = BCGSimulation
        self.honest, self.byzantine, self.max_rounds = honest, byzantine, max_rounds
        self.seed_base = seed * 100003 + replica * 7919
        self.lock = threading.Lock()
        self.generation = [0] * n_sims
        self.sims = [self._new_sim(i) for i in range(n_sims)]
        self.retired = 0          # accepted decisions of games already replaced
        self.retired_counters = {}  # every simulation counter of games already replaced
        self.games_finished = 0
        self.game_rounds = []     # rounds played by each finished game (burn-in rounds included)
        self.engine_rounds = []   # ... of them on the engine (burn-in rounds excluded)
        self.ages = [0] * n_sims  # burn-in rounds of each slot's first game
        self.outcomes = {}
        self.errors = []
        self._stop = threading.Event()
        self.threads = []

    def burn_in(self, p: float, seed: int, strategy_chars: int, reasoning_chars: int):
        """Age-diverse start: slot i's first game plays A_i ~ Geometric(p) rounds (support
        0, 1, 2, ...; capped below max_rounds) on a scripted CPU engine before the pool
        starts.  In a pool that has run for a long time a slot's game age is distributed
        as P(age >= a) = P(game length > a); with a per-round stop probability p that is
        this geometric law, so the timed windows see the round mix of whole games
        instead of every game in its first rounds at once.  Burn-in decisions are not
        counted (the counters are reset) and happen before warmup."""
        from byzantine_consensus_llm_agents_amd.engine.fake import BurnInLLM
        if p <= 0:
            return
        rng = random.Random(seed * 7919 + 17)
        fake = BurnInLLM(strategy_chars, reasoning_chars, seed)
        for i, sim in enumerate(self.sims):
            a = 0
            while rng.random() > p and a < self.max_rounds - 1:
                a += 1
            llms = {aid: ag.llm for aid, ag in sim.agents.items()}
            for ag in sim.agents.values():
                ag.llm = fake
            for _ in range(a):
                if sim.game.game_over:
                    break
                sim.run_round()
            for aid, ag in sim.agents.items():
                ag.llm = llms[aid]
            for k in sim.counters:
                sim.counters[k] = 0
            self.ages[i] = a

    def filled(self) -> bool:
        """Every slot's current game has completed at least one decide phase."""
        with self.lock:
            return all(s.counters["decisions_accepted"] > 0 or g > 0 for s, g in zip(self.sims, self.generation))

    def output_chars(self):
        """Mean public_reasoning / internal_strategy characters of the agents' latest outputs."""
        reason, strat = [], []
        with self.lock:
            for sim in self.sims:
                for ag in sim.agents.values():
                    reason.append(len(getattr(ag, "last_reasoning", "") or ""))
                    hist = getattr(ag.state, "last_k_internal_strategies", None)
                    if hist:
                        strat.append(len(hist[-1][1] if isinstance(hist[-1], tuple) else str(hist[-1])))
        mean = lambda v: round(sum(v) / len(v), 1) if v else None  # noqa: E731
        return {"public_reasoning": mean(reason), "internal_strategy": mean(strat)}

    def _new_sim(self, slot):
        seed = self.seed_base + slot * 1_000_003 + self.generation[slot]
        return self.BCGSimulation(self.honest, self.byzantine, config={
            "max_rounds": self.max_rounds, "value_range": (0, 50), "consensus_threshold": 66.0,
            "verbose": False, "byzantine_awareness": "may_exist", "seed": seed})

    @staticmethod
    def _made(sim) -> int:
        return sim.counters["decisions_accepted"] + sim.counters["votes_accepted"]

    def accepted(self) -> int:
        """Accepted decisions so far over every game this pool played (consistent snapshot)."""
        with self.lock:
            return self.retired + sum(self._made(s) for s in self.sims)

    def counter_totals(self) -> dict:
        """Every simulation counter (accepted outputs, retry-ladder calls, rows, exhausted
        outputs) summed over every game this pool played."""
        with self.lock:
            tot = dict(self.retired_counters)
            for s in self.sims:
                for k, v in s.counters.items():
                    tot[k] = tot.get(k, 0) + v
            return tot

    def _work(self, i, delay):
        try:
            if delay > 0 and self._stop.wait(delay):
                return
            while not self._stop.is_set():
                sim = self.sims[i]
                sim.run_round()
                if sim.game.game_over:
                    o = sim.game.get_statistics().get("consensus_outcome")
                    self.generation[i] += 1
                    fresh = self._new_sim(i)
                    with self.lock:
                        self.outcomes[o] = self.outcomes.get(o, 0) + 1
                        self.games_finished += 1
                        played = min(sim.game.current_round, sim.game.max_rounds)
                        self.game_rounds.append(played)
                        self.engine_rounds.append(played - (self.ages[i] if self.generation[i] == 1 else 0))
                        self.retired += self._made(sim)
                        for k, v in sim.counters.items():
                            self.retired_counters[k] = self.retired_counters.get(k, 0) + v
                        self.sims[i] = fresh
        except BaseException as exc:  # surfaced by the main thread
            self.errors.append(exc)

    def start(self, ramp_s: float = 0.0):
        n = len(self.sims)
        for i in range(n):
            delay = ramp_s * i / n if n > 1 else 0.0
            t = threading.Thread(target=self._work, args=(i, delay), name=f"sim{i}", daemon=True)
            self.threads.append(t)
            t.start()

    def stop(self):
        self._stop.set()

    def check(self):
        if self.errors:
            raise self.errors[0]


def window_stats(per_window, window_s: float):
    """Spread of the per-window decision counts: the naive standard error of the mean window
    (windows treated as independent) and the batch-means standard error over blocks of 4
    windows (a game's phase completions cluster, so neighbouring windows anti-correlate and the
    block estimate is the honest one for the run's total), both in % of the mean."""
    import statistics
    n = len(per_window)
    if n < 2 or sum(per_window) == 0:
        return {"n": n}
    mean = statistics.fmean(per_window)
    se = statistics.stdev(per_window) / n ** 0.5
    out = {"n": n, "mean": round(mean, 1), "sd": round(statistics.stdev(per_window), 1),
           "se_pct": round(100 * se / mean, 2)}
    blocks = [sum(per_window[i:i + 4]) / 4 for i in range(0, n - n % 4, 4)]
    if len(blocks) >= 2:
        out["block4_se_pct"] = round(100 * statistics.stdev(blocks) / len(blocks) ** 0.5 / mean, 2)
    return out


RETRY_KEYS = ("decide_prompts", "vote_prompts", "decide_batches", "vote_batches", "batch_rows",
              "sequential_calls", "sequential_attempts", "decisions_exhausted", "votes_exhausted")


def retry_summary(delta: dict) -> dict:
    """Timed-region cost of the retry ladder (retries count toward time, not toward
    decisions): prompts the games asked for, rows the engine generated for them (batch rows incl.
    re-batched failures + the agents' own sequential attempts), and outputs that exhausted every
    attempt.  `engine_rows_per_prompt` - 1 is the generation work retries added."""
    out = {k: int(delta.get(k, 0)) for k in RETRY_KEYS}
    prompts = out["decide_prompts"] + out["vote_prompts"]
    rows = out["batch_rows"] + out["sequential_attempts"]
    out["retry_rows"] = rows - prompts
    out["engine_rows_per_prompt"] = round(rows / prompts, 4) if prompts else None
    exhausted = out["decisions_exhausted"] + out["votes_exhausted"]
    out["exhausted_pct"] = round(100.0 * exhausted / prompts, 2) if prompts else None
    return out


def percentiles(values) -> dict:
    """n / p50 / p95 / max of a list of prompt lengths (tokens)."""
    if not values:
        return {"n": 0}
    v = sorted(values)
    pick = lambda q: v[min(len(v) - 1, int(q * (len(v) - 1) + 0.5))]  # noqa: E731
    return {"n": len(v), "p50": pick(0.50), "p95": pick(0.95), "max": v[-1]}


def thread_cpu():
    """{native thread id: (group, CPU seconds)} of this process's live threads.  Groups: the game
    threads (`sim*`), the engine's scheduler thread, the main thread, other Python threads, and
    threads with no Python name (HIP runtime, the tokenizer's rayon pool, gloo)."""
    try:
        import psutil
    except ImportError:
        return {}
    names = {t.native_id: t.name for t in threading.enumerate()}

    def native(tid):  # the OS thread name, its numeric suffix dropped: one group per pool
        try:
            with open(f"/proc/self/task/{tid}/comm") as f:
                return "native:" + (f.read().strip().rstrip("0123456789-_ ") or "?")
        except OSError:
            return "native"

    def group(name, tid):
        if name is None:
            return native(tid)
        if name.startswith("sim"):
            return "game_threads"
        if name.startswith("bcg-engine") or name.startswith("bcg-tp"):
            return "engine"
        return "main" if name == "MainThread" else "python_other"
    return {t.id: (group(names.get(t.id), t.id), t.user_time + t.system_time) for t in psutil.Process().threads()}


def thread_cpu_delta(before: dict, after: dict, total_s: float) -> dict:
    """CPU seconds per thread group between two `thread_cpu` snapshots; threads that ended in
    between (the short-lived sequential-retry threads) show up as `unattributed`."""
    out = {}
    for tid, (grp, t) in after.items():
        out[grp] = out.get(grp, 0.0) + t - before.get(tid, (grp, 0.0))[1]
    out = {k: round(v, 1) for k, v in sorted(out.items())}
    out["unattributed"] = round(total_s - sum(out.values()), 1)
    return out


from byzantine_consensus_llm_agents_amd.utils.threads import rank_thread_budget  # noqa: E402


def _heartbeat(llm, pool, stop: threading.Event, every: float = 30.0):
    """Progress line on stderr every `every` s (long runs must keep writing)."""
    t0 = time.perf_counter()
    while not stop.wait(every):
        st = dict(getattr(llm.backend, "stats", {}))
        print(f"[progress] {time.perf_counter() - t0:.0f}s accepted={pool.accepted()} {json.dumps(st)}",
              file=sys.stderr, flush=True)


def main(argv=None):
    args = parse(argv)
    world = int(os.environ.get("WORLD_SIZE", "0") or 0)
    if world == 0 and args.gpus > 1:
        sys.exit(self_launch(args))
    world = max(world, 1)
    if "BCG_BENCH_T0" in os.environ:  # self-launched rank: the deadline counts from the parent's start
        t0_wall = float(os.environ["BCG_BENCH_T0"])
        t_origin = time.perf_counter() - (time.time() - t0_wall)
    else:
        t_origin = T_PROCESS0
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    host_threads = rank_thread_budget(world)  # before torch / tokenizers start their pools
    if args.gpus != world and rank == 0:
        print(f"[bench] --gpus {args.gpus} but WORLD_SIZE={world}: measuring {world} rank(s)", file=sys.stderr)

    # stdout carries exactly ONE line (the JSON result): anything else -- e.g. the
    # reference's console messages when an agent fails all JSON retries, or native libraries
    # writing to fd 1 (gloo's "[Gloo] Rank ... connected" lines) -- goes to stderr
    sys.stdout.flush()
    result_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    sys.stdout = sys.stderr
    if os.environ.get("BCG_STACKS_AFTER"):  # debugging aid: dump every thread's stack periodically
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["BCG_STACKS_AFTER"]), repeat=True, file=sys.stderr)

    import torch
    import torch.distributed as dist
    torch.set_num_threads(min(torch.get_num_threads(), host_threads))

    gpu = args.backend == "hip"
    if args.backend == "hostmodel":
        os.environ.setdefault("BCG_HOSTMODEL_TOKENS_S", "34000")
    ctrl = None
    if args.one_device:
        local = 0
        os.environ["BCG_CUSTOM_AR"] = "force"
    if gpu:
        torch.cuda.set_device(local)
    if world > 1:
        import datetime
        dist.init_process_group("nccl" if gpu and not args.one_device else "gloo",
                                timeout=datetime.timedelta(seconds=900))
        # control plane (barriers, result reduction) on a CPU group: never queued on a
        # HIP stream behind the engine's kernels / TP collectives
        ctrl = dist.new_group(backend="gloo") if gpu and not args.one_device else dist.group.WORLD

    from byzantine_consensus_llm_agents_amd.bcg import config as C
    from byzantine_consensus_llm_agents_amd.bcg.engine_agent import EngineAgent
    from byzantine_consensus_llm_agents_amd.engine.llm import LLM
    from byzantine_consensus_llm_agents_amd.models.config import ALIASES

    model = ALIASES.get(args.model, args.model)
    replica = rank // args.tp
    C.METRICS_CONFIG["save_results"] = False
    C.VLLM_CONFIG["model_name"] = model
    C.VLLM_CONFIG["tensor_parallel_size"] = args.tp
    C.VLLM_CONFIG["quantization"] = args.quantization
    C.ENGINE_CONFIG.update(backend=args.backend, budget_aware_json=True, seed=args.seed + replica,
                           validity_aware_json=0 if args.plain_grammar else VALIDITY_MIN_VISIBLE,
                           ascii_text_json=not args.plain_grammar and not args.unicode_text,
                           use_hip_graphs=not args.no_graphs, prefix_caching=not args.no_prefix_cache,
                           custom_allreduce=not args.no_custom_allreduce,
                           kv_cache_dtype=args.kv_cache_dtype)
    if C.ENGINE_CONFIG.get("num_layers_override"):
        raise SystemExit("bench.py: num_layers_override (reduced depth) is a test option, never a measurement")
    if args.max_batch_seqs:
        C.ENGINE_CONFIG["max_batch_seqs"] = args.max_batch_seqs
    if args.kv_cache_gb:
        C.ENGINE_CONFIG["kv_cache_gb"] = args.kv_cache_gb
    C.BCG_CONFIG["value_range"] = (0, 50)
    random.seed(args.seed + rank)

    t0 = time.perf_counter()
    llm = LLM(model, max_model_len=C.VLLM_CONFIG["max_model_len"],
              gpu_memory_utilization=C.VLLM_CONFIG["gpu_memory_utilization"],
              tensor_parallel_size=args.tp, backend=args.backend, seed=args.seed + replica,
              quantization=args.quantization)
    # share the engine with every agent (same model name + config => no reload)
    EngineAgent._shared_llm = llm
    EngineAgent._shared_model_name = model
    EngineAgent._shared_model_config = dict(C.VLLM_CONFIG)
    init_s = time.perf_counter() - t0

    def barrier():
        if world > 1:
            dist.barrier(group=ctrl)

    from byzantine_consensus_llm_agents_amd.bcg.prompts import all_schemas
    llm.precompile(all_schemas(0, 50))  # every rank, same order: identical FSM row bases
    pool = None
    if llm.is_driver:
        llm.start_continuous_batching()
        pool = SimPool(args.sims_per_gpu, args.honest, args.byzantine, args.max_rounds, args.seed, replica)
        sc, rc = (int(x) for x in args.burnin_chars.split(","))
        t_b = time.perf_counter()
        pool.burn_in(args.age_p, args.seed + replica, sc, rc)
        if rank == 0:
            print(f"[burn-in] ages {sum(pool.ages) / len(pool.ages):.2f} rounds mean, max {max(pool.ages)} "
                  f"({time.perf_counter() - t_b:.1f}s)", file=sys.stderr, flush=True)
        ramp = args.ramp_s if args.ramp_s is not None else 0.5 * args.warmup * args.window_s
        pool.start(ramp_s=ramp)
    else:
        llm.start_worker()  # TP follower: executes the group driver's plans until it stops

    stop_hb = threading.Event()
    if rank == 0:
        threading.Thread(target=_heartbeat, args=(llm, pool, stop_hb), daemon=True).start()

    def accepted():
        if pool is None:
            return 0
        pool.check()
        return pool.accepted()

    # Pool fill (untimed, before the warmup windows): all games start within the ramp, so their
    # first prompts arrive as one prefill wave that a long-running pool never sees; wait until
    # every game has finished its first decide phase.  TP followers / other DP ranks wait at the
    # barrier below.
    t_fill = time.perf_counter()
    if pool is not None:
        deadline_fill = t_fill + args.fill_max_s
        while time.perf_counter() < deadline_fill and not pool.filled():
            pool.check()
            time.sleep(0.5)
    fill_s = time.perf_counter() - t_fill
    barrier()
    # W warmup windows of pool time: a fill that already ran that long counts toward them
    time.sleep(max(0.0, args.window_s * args.warmup - fill_s))
    if rank == 0:
        print(f"[warmup] fill {fill_s:.1f}s, warmup {max(fill_s, args.warmup * args.window_s):.1f}s "
              f"(>= {args.warmup} x {args.window_s}s windows), accepted={accepted()} "
              f"init={init_s:.1f}s", file=sys.stderr, flush=True)

    eng = getattr(llm.backend, "stats", {})
    stats0 = dict(eng)
    plens = getattr(llm.backend, "prompt_lens", None)
    plen0 = {k: len(v) for k, v in plens.items()} if plens is not None else None
    barrier()
    if gpu:
        torch.cuda.synchronize()
    t_start = time.perf_counter()
    cpu0 = time.process_time()  # this rank's host CPU (all threads) over the timed region
    thr0 = thread_cpu()
    sampler = None
    if os.environ.get("BCG_HOST_SAMPLE") == "1":  # where the host CPU goes (utils/host_sampler.py)
        from byzantine_consensus_llm_agents_amd.utils.host_sampler import HostSampler
        sampler = HostSampler().start()
    ctr0 = pool.counter_totals() if pool is not None else {}
    a0 = accepted()
    per_window, steps_done, last = [], 0, a0

    def eng_tokens():  # uncached prompt + generated tokens so far (the engine's live counters)
        return eng.get("prompt_tokens", 0) - eng.get("cached_tokens", 0) + eng.get("generated_tokens", 0)

    tok_windows, tok_last = [], eng_tokens()
    # the deadline is agreed on by every rank (the slowest start wins)
    budget = torch.tensor([args.deadline_s - (t_start - t_origin)], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(budget, op=dist.ReduceOp.MIN, group=ctrl)
    max_windows = max(1, min(args.steps, int(float(budget[0]) // args.window_s)))
    for k in range(max_windows):
        delay = t_start + (k + 1) * args.window_s - time.perf_counter()
        if delay > 0:
            time.sleep(delay)
        now = accepted()
        per_window.append(now - last)
        last = now
        t_now = eng_tokens()
        tok_windows.append(t_now - tok_last)
        tok_last = t_now
        steps_done += 1
    decisions = last - a0
    ctr1 = pool.counter_totals() if pool is not None else {}
    if gpu:
        torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t_start
    # (bookkeeping after the clock stops: none of it inside the timed region)
    host_cpu_s = time.process_time() - cpu0
    threads_cpu = thread_cpu_delta(thr0, thread_cpu(), host_cpu_s)
    host_samples = sampler.stop() if sampler is not None else None
    retry_delta = [float(ctr1.get(k, 0) - ctr0.get(k, 0)) for k in RETRY_KEYS]
    if rank == 0:
        print(f"[timed] {steps_done} windows decisions={decisions} elapsed={elapsed:.2f}s", file=sys.stderr,
              flush=True)

    # DP replicas: only the group driver's pool counts (TP followers run no games)
    if world > 1:
        t = torch.tensor([float(decisions), elapsed], dtype=torch.float64)
        tot, mx = t[:1].clone(), t[1:].clone()
        dist.all_reduce(tot, op=dist.ReduceOp.SUM, group=ctrl)
        dist.all_reduce(mx, op=dist.ReduceOp.MAX, group=ctrl)
        total_decisions, elapsed = float(tot[0]), float(mx[0])
    else:
        total_decisions = float(decisions)
    value = total_decisions / elapsed if elapsed > 0 else 0.0
    d_eng = {k: eng.get(k, 0) - stats0.get(k, 0) for k in eng}
    # engine token rate of the timed region (uncached prompt + generated tokens), summed over DP
    # replicas: the smooth companion of the bursty decision count (a game's 10 agents finish a
    # phase together), used for A/B comparisons
    tok = float(d_eng.get("prompt_tokens", 0) - d_eng.get("cached_tokens", 0) + d_eng.get("generated_tokens", 0))
    if pool is None:
        tok = 0.0  # TP followers: their driver counts the group's tokens
    if world > 1:
        tt = torch.tensor([tok], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.SUM, group=ctrl)
        tok = float(tt[0])
    tokens_per_s = tok / elapsed if elapsed > 0 else 0.0
    if world > 1:  # retry-ladder counters summed over the DP replicas' pools
        rt = torch.tensor(retry_delta, dtype=torch.float64)
        dist.all_reduce(rt, op=dist.ReduceOp.SUM, group=ctrl)
        retry_delta = rt.tolist()
    retry = retry_summary(dict(zip(RETRY_KEYS, retry_delta)))
    # prompt sizes of the timed region per phase (the engine records them by requested max_tokens)
    phase_of = {C.LLM_CONFIG["max_tokens_decide"]: "decide", C.LLM_CONFIG["max_tokens_vote"]: "vote"}
    prompt_tokens = None
    if plens is not None:
        prompt_tokens = {}
        for mt, lens in list(plens.items()):
            name = phase_of.get(mt, f"max_tokens_{mt}")
            prompt_tokens.setdefault(name, []).extend(lens[plen0.get(mt, 0):])
        prompt_tokens = {k: percentiles(v) for k, v in sorted(prompt_tokens.items())}
    context = {"rejects": int(d_eng.get("context_rejects", 0)), "short": int(d_eng.get("context_short", 0)),
               "max_model_len": C.VLLM_CONFIG["max_model_len"]}
    # the layout as every rank saw it: which ranks drive a game pool (one per DP replica, its own
    # seeds) and which only execute their TP driver's plans
    me = {"rank": rank, "replica": replica, "driver": pool is not None,
          "seed_base": pool.seed_base if pool is not None else None,
          "sims": len(pool.sims) if pool is not None else 0, "decisions": decisions if pool is not None else 0}
    ranks = [me]
    if world > 1:
        ranks = [None] * world
        dist.all_gather_object(ranks, me, group=ctrl)
    # host budget: CPU seconds of every rank's process over the timed region (summed) and the
    # slowest DP replica's decision rate
    per_rank_rate = decisions / elapsed if elapsed > 0 and pool is not None else float("inf")
    if world > 1:
        hc = torch.tensor([host_cpu_s], dtype=torch.float64)
        dist.all_reduce(hc, op=dist.ReduceOp.SUM, group=ctrl)
        host_cpu_s = float(hc[0])
        mr = torch.tensor([per_rank_rate], dtype=torch.float64)
        dist.all_reduce(mr, op=dist.ReduceOp.MIN, group=ctrl)
        per_rank_rate = float(mr[0])
    stats = window_stats(per_window, args.window_s)
    tp_status = getattr(getattr(llm.backend, "tp", None), "custom_status", "off") if args.tp > 1 else "off"
    if world > 1:  # every group agrees on its own status; rank 0 reports the first fallback, if any
        statuses = [None] * world
        dist.all_gather_object(statuses, tp_status, group=ctrl)
        tp_status = next((s for s in statuses if s.startswith("fallback")), statuses[0])
    if rank == 0:
        line = {
            "metric": f"agent decisions/sec (node), {args.honest}h+{args.byzantine}b BCG {model.split('/')[-1]}; "
                      "consensus-rate parity",
            "value": round(value, 3), "unit": "decisions/s", "n_gpus": world, "steps": steps_done,
            "warmup": args.warmup, "ms_per_step": round(1000 * elapsed / max(steps_done, 1), 2),
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": (value / BASELINE_VALUE) if BASELINE_VALUE else None,
            "dtype": "fp8" if args.quantization == "fp8" else "bf16",
            "kv_cache_dtype": "fp8" if args.kv_cache_dtype == "fp8" else "bf16",
            "data": "synthetic (random-init weights, synthetic BPE tokenizer, budget-aware JSON grammar"
                    + ("" if args.plain_grammar else f", validity-aware: every field, >= {VALIDITY_MIN_VISIBLE} "
                       "visible chars per free-text field"
                       + ("" if args.unicode_text else ", printable-ASCII free text")) + ")",
            "config": {"model": model, "honest": args.honest, "byzantine": args.byzantine,
                       "global_batch": args.sims_per_gpu * (args.honest + args.byzantine) * (world // args.tp),
                       "sims_per_gpu": args.sims_per_gpu, "seq_len": C.VLLM_CONFIG["max_model_len"],
                       "max_batch_seqs": C.ENGINE_CONFIG["max_batch_seqs"],
                       "max_tokens_decide": C.LLM_CONFIG["max_tokens_decide"],
                       "max_tokens_vote": C.LLM_CONFIG["max_tokens_vote"],
                       "max_rounds": args.max_rounds, "age_p": args.age_p,
                       "step": f"{args.window_s:g} s window of the continuously-batched pool",
                       "parallelism": f"dp{world // args.tp}" + (f"xtp{args.tp}" if args.tp > 1 else ""),
                       "hip_graphs": not args.no_graphs and getattr(llm.backend, "graphs_off_reason", None) is None,
                       "prefix_caching": not args.no_prefix_cache,
                       "poll_every": C.ENGINE_CONFIG.get("poll_every"),
                       "admit_max_wait": C.ENGINE_CONFIG.get("admit_max_wait"),
                       "prefill_carry_bursts": C.ENGINE_CONFIG.get("prefill_carry_bursts"),
                       "grammar": "budget-aware" + ("" if args.plain_grammar else
                                                    f" + validity-aware({VALIDITY_MIN_VISIBLE})"
                                                    + ("" if args.unicode_text else " + ascii-text")),
                       # "on" (xGMI kernels, cross-checked at init), "off", or "fallback:<reason>"
                       "custom_allreduce": tp_status},
            "detail": {"decisions": total_decisions, "elapsed_s": round(elapsed, 3), "init_s": round(init_s, 1),
                       "steps_requested": args.steps, "window_s": args.window_s,
                       "decisions_per_window_rank0": per_window,
                       "first5_vs_last5": [round(sum(per_window[:5]) / max(1, len(per_window[:5])), 1),
                                           round(sum(per_window[-5:]) / max(1, len(per_window[-5:])), 1)],
                       "fill_s": round(fill_s, 1), "fill_max_s": args.fill_max_s,
                       "fill_capped": fill_s >= args.fill_max_s - 0.5,
                       "tokens_per_s": round(tokens_per_s, 1), "window_stats_rank0": stats,
                       # the same spread for the engine's token count per window: the smooth
                       # series A/B comparisons should use
                       "token_window_stats_rank0": window_stats(tok_windows, args.window_s),
                       "retry": retry,
                       "prompt_tokens_rank0": prompt_tokens, "context_rank0": context,
                       "ranks": ranks,
                       "host": {"cpu_s_all_ranks": round(host_cpu_s, 1),
                                # rank 0's CPU seconds by thread group over the timed region
                                "cpu_s_by_thread_rank0": threads_cpu,
                                **({"samples_rank0": host_samples} if host_samples else {}),
                                "threads_per_rank": host_threads,
                                "rayon_threads": os.environ.get("RAYON_NUM_THREADS"),
                                "cpu_s_per_decision": (round(host_cpu_s / total_decisions, 4)
                                                       if total_decisions else None),
                                "min_replica_decisions_per_s": round(per_rank_rate, 3),
                                "host_cpus": os.cpu_count()},
                       "age_mix": {"p": args.age_p, "burnin_chars": args.burnin_chars,
                                   "mean_burnin_rounds": (round(sum(pool.ages) / len(pool.ages), 2)
                                                          if pool else None),
                                   "mean_rounds_per_finished_game": (
                                       round(sum(pool.game_rounds) / len(pool.game_rounds), 2)
                                       if pool and pool.game_rounds else None),
                                   # rounds each finished game played on the engine (its burn-in
                                   # rounds on the scripted CPU engine excluded)
                                   "mean_engine_rounds_per_finished_game": (
                                       round(sum(pool.engine_rounds) / len(pool.engine_rounds), 2)
                                       if pool and pool.engine_rounds else None),
                                   "protocol": ("burn-in (age-mixed pool, first games aged on a scripted "
                                                "CPU engine)" if args.age_p > 0 else "fresh pool"),
                                   "output_chars": pool.output_chars() if pool else None},
                       "engine_per_rank": d_eng, "games_finished_rank0": pool.games_finished if pool else 0,
                       "outcomes_rank0": pool.outcomes if pool else {},
                       "wall_since_start_s": round(time.perf_counter() - t_origin, 1),
                       "phases_rank0": llm.backend.timer.summary() if hasattr(llm.backend, "timer") else {}},
        }
        print(json.dumps(line), file=result_out, flush=True)
    stop_hb.set()
    if pool is not None:
        pool.stop()
    # game threads still waiting on the engine are daemons: they die with the process
    llm.shutdown()
    if world > 1:
        barrier()
        from byzantine_consensus_llm_agents_amd.parallel import groups
        groups.destroy()  # custom all-reduce buffers unmapped while every peer is still alive
        # skip interpreter finalization: a daemon game thread unwound inside native code
        # there (pthread_exit through a noexcept frame) aborts the rank after its result is out
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)


if __name__ == "__main__":
    main()
