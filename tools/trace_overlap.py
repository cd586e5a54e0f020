"""Summarise a rocprofv3 kernel trace: per-queue busy time, cross-queue overlap, GPU idle.

  python tools/trace_overlap.py gpurun_out/prof/run_kernel_trace.csv.gz [--top 15]

Used to check that prefill (its own HIP stream) really runs concurrently with
the decode graph replays, and how much of the wall time the GPU sits idle.
"""
import argparse
import collections
import csv
import gzip
import json
import sys

csv.field_size_limit(sys.maxsize)


def short(name: str) -> str:
    name = name.split("(")[0]
    return name[-60:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--top", type=int, default=12)
    ap.add_argument("--window", type=float, default=0.0, help="also print GPU idle %% per window of this many s")
    a = ap.parse_args()
    opener = gzip.open if a.trace.endswith(".gz") else open
    ev = []
    with opener(a.trace, "rt") as fh:
        for row in csv.DictReader(fh):
            ev.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), int(row["Queue_Id"]),
                       short(row["Kernel_Name"])))
    ev.sort()
    t0, t1 = ev[0][0], max(e[1] for e in ev)
    per_q = collections.defaultdict(int)
    per_q_names = collections.defaultdict(collections.Counter)
    for s, e, q, n in ev:
        per_q[q] += e - s
        per_q_names[q][n] += e - s
    # union of busy intervals (all queues) and time with >=2 queues busy
    points = []
    for s, e, q, _ in ev:
        points.append((s, 1, q))
        points.append((e, -1, q))
    points.sort()
    active = collections.Counter()
    busy = both = 0
    last = points[0][0]
    for t, d, q in points:
        nq = sum(1 for v in active.values() if v > 0)
        if nq >= 1:
            busy += t - last
        if nq >= 2:
            both += t - last
        active[q] += d
        last = t
    out = {"wall_ms": (t1 - t0) / 1e6, "busy_ms": busy / 1e6, "idle_ms": (t1 - t0 - busy) / 1e6,
           "multi_queue_ms": both / 1e6,
           "queues": {q: {"busy_ms": v / 1e6,
                          "top": [(n, round(t / 1e6, 1)) for n, t in per_q_names[q].most_common(a.top)]}
                      for q, v in sorted(per_q.items())}}
    print(json.dumps(out, indent=1))
    if a.window > 0:
        w = int(a.window * 1e9)
        nwin = (t1 - t0) // w + 1
        busy_w = [0] * nwin
        # merge intervals, then spread the busy time over windows
        cur_s, cur_e = ev[0][0], ev[0][1]
        merged = []
        for s, e, _, _ in ev[1:]:
            if s <= cur_e:
                cur_e = max(cur_e, e)
            else:
                merged.append((cur_s, cur_e))
                cur_s, cur_e = s, e
        merged.append((cur_s, cur_e))
        for s, e in merged:
            while s < e:
                k = (s - t0) // w
                edge = t0 + (k + 1) * w
                busy_w[k] += min(e, edge) - s
                s = min(e, edge)
        print("idle % per window:", " ".join(f"{100 - 100 * b / w:.0f}" for b in busy_w))


if __name__ == "__main__":
    main()
