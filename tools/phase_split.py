"""Split a rocprofv3 kernel trace of the engine into prefill and decode GPU time, per kernel family.

  python tools/phase_split.py gpurun_out/prof/run_kernel_trace.csv.gz [--skip-s 60]

Every decoder layer launches its kernels in a fixed order around ONE attention kernel
(prefill: ``prefill_attn_kernel``; decode: ``decode_attn_kernel`` with its shared-prefix and
combine kernels), so a kernel between two attention kernels of the same mode belongs to
that mode.  At a mode switch the kernels from the new layer's input norm on (norm, qkv GEMM, QK-norm +
RoPE + KV write, shared-prefix pass) go to the new mode, the rest to the old one.
Kernels outside any forward (sampler, state updates) are counted under the mode of the
surrounding attention kernels as well; their time is small.  ``--skip-s`` drops the first
seconds of the trace (start-up: model init, graph capture, the fill wave).
"""
import argparse
import collections
import csv
import gzip
import json
import sys

csv.field_size_limit(sys.maxsize)

FAMILIES = [  # (substring of the kernel name, family); first match wins
    ("decode_shared_kernel", "attn_decode_shared"), ("decode_attn_kernel", "attn_decode"),
    ("decode_combine_kernel", "attn_decode_combine"), ("prefill_attn", "attn_prefill"),
    ("gemm_w4_kernel", "gemm_hand_w4"), ("gemm_pp_kernel", "gemm_hand_256x256"), ("gemm_nt_kernel", "gemm_hand_tiles"),
    ("Cijk_", "gemm_hipblaslt"),
    ("qk_norm_rope", "rope_kv"), ("rmsnorm", "norm"), ("silu_mul", "silu_mul"), ("sample", "sampler"),
]


def family(name: str) -> str:
    for key, fam in FAMILIES:
        if key in name:
            return fam
    return "other"


def attn_mode(name: str):
    if "prefill_attn" in name:
        return "prefill"
    if "decode_attn_kernel" in name:
        return "decode"
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip-s", type=float, default=0.0)
    a = ap.parse_args()
    opener = gzip.open if a.trace.endswith(".gz") else open
    ev = []
    with opener(a.trace, "rt") as fh:
        for row in csv.DictReader(fh):
            ev.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]), row["Kernel_Name"]))
    ev.sort()
    t_skip = ev[0][0] + int(a.skip_s * 1e9)
    ev = [e for e in ev if e[0] >= t_skip]
    modes = [None] * len(ev)
    attn_idx = [i for i, e in enumerate(ev) if attn_mode(e[2])]
    for j, i in enumerate(attn_idx):
        m = attn_mode(ev[i][2])
        modes[i] = m
        prev = attn_idx[j - 1] if j else -1
        pm = attn_mode(ev[prev][2]) if prev >= 0 else m
        cut = prev + 1  # at a switch: the new mode starts at the layer's input norm
        if pm != m:
            cut = next((k for k in range(i - 1, prev, -1) if family(ev[k][2]) == "norm"), max(prev + 1, i - 3))
        for k in range(prev + 1, i):
            modes[k] = m if k >= cut else pm
    last = attn_mode(ev[attn_idx[-1]][2]) if attn_idx else "decode"
    for k in range((attn_idx[-1] + 1) if attn_idx else 0, len(ev)):
        modes[k] = last
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    for (s, e, n), m in zip(ev, modes):
        tot[m][family(n)] += (e - s) / 1e6
    wall = (ev[-1][1] - ev[0][0]) / 1e6
    busy = sum(sum(v.values()) for v in tot.values())
    out = {"wall_ms": round(wall, 1), "kernel_ms": round(busy, 1), "skip_s": a.skip_s}
    for m in ("prefill", "decode"):
        fam = tot.get(m, {})
        sm = sum(fam.values())
        out[m] = {"ms": round(sm, 1), "share_of_kernel_time": round(sm / busy, 4) if busy else 0,
                  "families_ms": {k: round(v, 1) for k, v in sorted(fam.items(), key=lambda x: -x[1])}}
    out["decode_steps_approx"] = sum(1 for i in attn_idx if attn_mode(ev[i][2]) == "decode") // 40 or None
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
