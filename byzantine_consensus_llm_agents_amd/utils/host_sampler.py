"""Where a rank's host CPU goes: a low-rate sampler of the engine thread's Python stack and of
every OS thread's run state (bench.py, env BCG_HOST_SAMPLE=1).

`time.thread_time` per thread says how much CPU each thread used, not on what.  This samples,
every `interval` seconds:

* the engine scheduler thread's Python stack (`sys._current_frames`): its innermost frame and
  the innermost frame inside this package -- a thread that burns CPU inside a C call (a HIP
  synchronize, a graph replay, a tokenizer call) shows the Python line that made the call;
* every OS thread's state from /proc/self/task/*/stat: R (running or runnable) samples per
  thread name (a native pool spinning shows up as R on every sample).
"""

import collections
import os
import sys
import threading
import time
from typing import Dict, Optional

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _frame_label(frame) -> str:
    code = frame.f_code
    return f"{os.path.basename(code.co_filename)}:{code.co_name}:{frame.f_lineno}"


def _pkg_frame(frame) -> Optional[str]:
    while frame is not None:
        if frame.f_code.co_filename.startswith(_PKG):
            return _frame_label(frame)
        frame = frame.f_back
    return None


def _task_states() -> Dict[str, str]:
    """{tid: (comm, state)} of this process's OS threads."""
    out = {}
    base = "/proc/self/task"
    try:
        tids = os.listdir(base)
    except OSError:
        return out
    for tid in tids:
        try:
            with open(f"{base}/{tid}/stat") as f:
                stat = f.read()
        except OSError:
            continue
        # pid (comm) state ...: comm may contain spaces, it ends at the last ')'
        lp, rp = stat.find("("), stat.rfind(")")
        out[tid] = (stat[lp + 1:rp], stat[rp + 2:rp + 3])
    return out


class HostSampler:
    def __init__(self, interval: float = 0.02, thread_prefix: str = "bcg-engine"):
        self.interval = interval
        self.thread_prefix = thread_prefix
        self.samples = 0
        self.engine_inner = collections.Counter()
        self.engine_pkg = collections.Counter()
        self.running = collections.Counter()  # thread name -> R samples
        self.threads = collections.Counter()  # thread name -> thread count (max seen)
        self.native_tid = collections.Counter()  # native thread id -> R samples (unnamed threads)
        self._stop = threading.Event()
        self._thread = None

    def start(self):
        self._thread = threading.Thread(target=self._run, name="bcg-host-sampler", daemon=True)
        self._thread.start()
        return self

    def _run(self):
        me = threading.get_ident()
        while not self._stop.wait(self.interval):
            self.samples += 1
            names = {t.ident: t.name for t in threading.enumerate()}
            native_names = {t.native_id: t.name for t in threading.enumerate()}
            for ident, frame in sys._current_frames().items():
                if ident == me or not names.get(ident, "").startswith(self.thread_prefix):
                    continue
                self.engine_inner[_frame_label(frame)] += 1
                self.engine_pkg[_pkg_frame(frame) or "?"] += 1
            per_name = collections.Counter()
            for tid, (comm, state) in _task_states().items():
                name = native_names.get(int(tid)) or f"native:{comm.rstrip('0123456789-_ ')}"
                if name.startswith("sim"):
                    name = "sim*"
                per_name[name] += 1
                if state == "R":
                    self.running[name] += 1
                    if name.startswith("native:"):
                        self.native_tid[tid] += 1
            for k, v in per_name.items():
                self.threads[k] = max(self.threads[k], v)

    @staticmethod
    def _describe(tid: str) -> Dict:
        """What a native thread is doing: its syscall (number, or 'running' in user space) and the
        kernel function it sleeps in."""
        out = {}
        for key in ("syscall", "wchan"):
            try:
                with open(f"/proc/self/task/{tid}/{key}") as f:
                    out[key] = f.read().split()[0] if key == "syscall" else f.read().strip()
            except (OSError, IndexError):
                pass
        return out

    def stop(self) -> Dict:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
        n = max(1, self.samples)
        busiest = [(tid, self._describe(tid)) for tid, v in self.native_tid.most_common(3) if v > 0.5 * n]
        top = lambda c, k=12: [(name, round(v / n, 3)) for name, v in c.most_common(k)]  # noqa: E731
        return {"samples": self.samples, "interval_s": self.interval,
                "engine_innermost": top(self.engine_inner), "engine_in_package": top(self.engine_pkg),
                # mean number of that name's threads in state R per sample (~ cores busy)
                "running_threads": top(self.running, 16), "thread_counts": dict(self.threads.most_common(16)),
                # the busiest unnamed threads one by one: a few at ~1.0 = spinning runtime threads,
                # many at a few % = a worker pool
                "native_busiest": [round(v / n, 3) for _, v in self.native_tid.most_common(24)],
                "native_spinning": [d for _, d in busiest]}
