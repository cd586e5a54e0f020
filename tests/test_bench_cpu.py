"""bench.py driver contract on CPU: torchrun with 2 gloo ranks and the fake engine.

Checks the one-JSON-line stdout contract the round driver parses (metric/value/unit,
n_gpus, steps, warmup, config.parallelism) and that the whole-job value sums the
DP replicas' decisions while TP peers contribute once (bench.py:216-226).
"""

import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config"}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(extra):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--backend", "fake", "--sims-per-gpu", "2"] + extra
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    p = subprocess.run(cmd, cwd="/tmp", env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    # gloo's C++ connection log ("[Gloo] Rank r is connected to ...", both ranks interleaved)
    # goes to the process's stdout below Python; RCCL prints nothing there.  Every JSON
    # line counts: exactly one (rank 0's) must exist.
    lines = [ln for ln in p.stdout.splitlines() if ln.lstrip().startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


@pytest.mark.parametrize("tp,parallelism,replicas", [(1, "dp2", 2), (2, "dp1xtp2", 1)])
def test_bench_two_ranks(tp, parallelism, replicas):
    out = _run(["--tp", str(tp), "--honest", "4", "--byzantine", "1"])
    assert KEYS <= set(out)
    assert out["n_gpus"] == 2 and out["steps"] == 2 and out["warmup"] == 1
    assert out["unit"] == "decisions/s" and out["higher_is_better"] is True and out["scaling"] == "weak"
    assert out["config"]["parallelism"] == parallelism
    assert out["config"]["global_batch"] == 2 * 5 * replicas
    # each simulation makes one decide + one vote per agent per round
    assert out["detail"]["decisions"] == replicas * 2 * 5 * 2 * 2
    assert out["value"] > 0 and out["ms_per_step"] > 0
