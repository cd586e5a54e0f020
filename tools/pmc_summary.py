"""Average each PMC counter per kernel over the rocprofv3 counter_collection CSVs under a directory."""
import collections
import csv
import glob
import os
import sys

csv.field_size_limit(sys.maxsize)


def main(root):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "?")
                name = name[5:] if name.startswith("void ") else name
                name = name.replace("(anonymous namespace)::", "").split("(")[0][:70]
                acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for name, counters in sorted(acc.items()):
        print(name)
        mean = {}
        for c, vals in sorted(counters.items()):
            mean[c] = sum(vals) / len(vals)
            print(f"    {c:36s} n={len(vals):5d} mean={mean[c]:16.1f}")
        if mean.get("SQ_INSTS_MFMA"):
            print(f"    VALU per MFMA instruction           {mean.get('SQ_INSTS_VALU', 0.0) / mean['SQ_INSTS_MFMA']:16.2f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
