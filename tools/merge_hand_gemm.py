"""Merge tuned hand-GEMM tables (tools/tune_hand_gemm.py --out ...) into the shipped one.

  python tools/merge_hand_gemm.py gpurun_out/hand_gemm_qwen3-8b_tp1.json gpurun_out/hand_gemm_qwen3-32b_tp4.json

Entries are keyed by (M, N, K, epilogue); a merged file's entry replaces the shipped one.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TABLE = os.path.join(ROOT, "byzantine_consensus_llm_agents_amd", "engine", "tuned", "hand_gemm.json")


def main(paths):
    with open(TABLE) as fh:
        table = json.load(fh)
    for path in paths:
        with open(path) as fh:
            add = json.load(fh)
        for part in ("choice", "timings_us"):
            table.setdefault(part, {}).update(add.get(part, {}))
        print(f"{path}: {len(add.get('choice', {}))} entries")
    with open(TABLE, "w") as fh:
        json.dump(table, fh, indent=1, sort_keys=True)
    print(f"{TABLE}: {len(table['choice'])} entries")


if __name__ == "__main__":
    main(sys.argv[1:])
