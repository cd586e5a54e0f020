"""Per-rank host thread budget: bench.py and bcg/sweep.py call it before
torch or the tokenizer start their pools.  No torch import here."""

import os


def rank_thread_budget(world: int) -> int:
    """Host threads per rank for the tokenizer's rayon pool, OpenMP and torch's CPU ops: this
    process's CPUs split over the node's ranks (without it every rank's pools default to every
    logical CPU of the node).  An explicit RAYON_NUM_THREADS / OMP_NUM_THREADS in the environment
    wins."""
    try:
        cpus = len(os.sched_getaffinity(0))
    except AttributeError:
        cpus = os.cpu_count() or 8
    local = int(os.environ.get("LOCAL_WORLD_SIZE", world) or world)
    per = max(2, min(16, cpus // max(1, local)))
    os.environ.setdefault("RAYON_NUM_THREADS", str(per))
    os.environ.setdefault("OMP_NUM_THREADS", str(per))
    os.environ.setdefault("TOKENIZERS_PARALLELISM", "true")
    return per
