"""Merge tools/bench_fp8_gemm.py timings into engine/tuned/hand_gemm_fp8.json (best per shape).

  python tools/merge_fp8_table.py gpurun_out/bench_fp8_gemm_tp2.json
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TABLE = os.path.join(ROOT, "byzantine_consensus_llm_agents_amd", "engine", "tuned", "hand_gemm_fp8.json")


def main(paths):
    with open(TABLE) as fh:
        table = json.load(fh)
    for path in paths:
        with open(path) as fh:
            timings = json.load(fh)
        for key, t in timings.items():
            best = min((v, k) for k, v in t.items())[1]
            table["choice"][key] = [-1, 1] if best == "lib" else [int(x) for x in best.split("x")]
        print(f"{path}: {len(timings)} shapes")
    with open(TABLE, "w") as fh:
        json.dump(table, fh, indent=1, sort_keys=True)
    print(f"{TABLE}: {len(table['choice'])} entries")


if __name__ == "__main__":
    main(sys.argv[1:])
