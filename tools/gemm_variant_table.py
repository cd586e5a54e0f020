"""Summarise tools/gpu_gemm_variants.sh output: best TF/s per (variant, shape) over the rounds."""
import collections
import json
import sys

rows = [json.loads(l) for l in open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/gemmv/times.jsonl")
        if l.startswith("{")]
best = collections.defaultdict(dict)
for r in rows:
    key = f"{r['M']}x{r['N']}x{r['K']} e{r['epi']} s{r['split']}"
    best[key][r["variant"]] = max(best[key].get(r["variant"], 0.0), r["tflops"])
variants = sorted({r["variant"] for r in rows})
print(f"{'shape':32s}" + "".join(f"{v:>12s}" for v in variants))
for key, vals in best.items():
    print(f"{key:32s}" + "".join(f"{vals.get(v, 0):12.0f}" for v in variants))
