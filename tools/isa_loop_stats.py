"""Instruction mix of the MFMA loop(s) of each kernel in a hipcc -S output (.s).

usage: python tools/isa_loop_stats.py kernel.s [name-substring]
Prints, per kernel, per loop (a backward branch target containing v_mfma): counts of
MFMA / ds_read / ds_write / buffer|global loads / s_waitcnt / scratch (spill) ops / barriers.
"""
import re
import sys
from collections import Counter


def kernels(text):
    for m in re.finditer(r"^(\S+):\s*; @\1\n(.*?)^\.Lfunc_end\d+:", text, re.M | re.S):
        yield m.group(1), m.group(2)


def classify(ins):
    op = ins.split()[0]
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("ds_read") or op.startswith("ds_load"):
        return "ds_read"
    if op.startswith("ds_write") or op.startswith("ds_store"):
        return "ds_write"
    if op.startswith("buffer_load") or op.startswith("global_load"):
        return "vmem_load"
    if op.startswith("buffer_store") or op.startswith("global_store"):
        return "vmem_store"
    if op.startswith("scratch_"):
        return "scratch"
    if op == "s_waitcnt":
        return "waitcnt"
    if op == "s_barrier":
        return "barrier"
    if op.startswith("v_accvgpr"):
        return "accvgpr"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    text = open(sys.argv[1]).read()
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    for name, body in kernels(text):
        if sub not in name:
            continue
        lines = [l.strip() for l in body.split("\n")]
        labels = {l.split(":")[0]: i for i, l in enumerate(lines) if re.match(r"^\.LBB\d+_\d+:", l)}
        print(name)
        for i, l in enumerate(lines):
            m = re.match(r"^s_cbranch_\w+\s+(\.LBB\d+_\d+)", l) or re.match(r"^s_branch\s+(\.LBB\d+_\d+)", l)
            if m and m.group(1) in labels and labels[m.group(1)] < i:
                seg = [x for x in lines[labels[m.group(1)]:i + 1] if x and not x.startswith((";", "."))]
                c = Counter(classify(x) for x in seg)
                if c["mfma"]:
                    print(f"  loop {m.group(1)} lines {labels[m.group(1)]}-{i}: " +
                          " ".join(f"{k}={v}" for k, v in sorted(c.items())))


if __name__ == "__main__":
    main()
