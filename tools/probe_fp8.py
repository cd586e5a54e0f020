"""Probe hipBLASLt fp8 (e4m3fn, OCP) GEMM support through torch._scaled_mm on gfx950.

  python tools/probe_fp8.py

Checks per-tensor and row-wise scaling, accuracy against a bf16 GEMM of the
dequantised operands, and times Mistral-Small-22B projection shapes against
bf16 F.linear.  Writes gpurun_out/probe_fp8.json.
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    out = {"device": torch.cuda.get_device_name(0), "results": []}
    f8 = torch.float8_e4m3fn
    shapes = {"qkv": (8192, 6144), "o": (6144, 6144), "gate_up": (32768, 6144), "down": (6144, 16384)}
    for M in (16, 128, 256, 8192):
        for name, (N, K) in shapes.items():
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
            sw = w.abs().amax(dim=1, keepdim=True).float() / 448.0
            sx = x.abs().amax(dim=1, keepdim=True).float() / 448.0
            wq = (w / sw).to(f8)
            xq = (x / sx).to(f8)
            ref = (xq.float() * sx) @ (wq.float() * sw).t()
            rec = {"M": M, "op": name, "N": N, "K": K}
            for mode in ("tensor", "rowwise"):
                try:
                    if mode == "tensor":
                        a_s, b_s = sx.max().reshape(()), sw.max().reshape(())
                        xq2, wq2 = (x / a_s).to(f8), (w / b_s).to(f8)
                        fn = lambda: torch._scaled_mm(xq2, wq2.t(), scale_a=a_s, scale_b=b_s,  # noqa: E731
                                                      out_dtype=torch.bfloat16)
                        ref2 = (xq2.float() * a_s) @ (wq2.float() * b_s).t()
                    else:
                        fn = lambda: torch._scaled_mm(xq, wq.t(), scale_a=sx, scale_b=sw.t(),  # noqa: E731
                                                      out_dtype=torch.bfloat16)
                        ref2 = ref
                    y = fn()
                    err = ((y.float() - ref2).norm() / ref2.norm()).item()
                    rec[f"{mode}_relerr"] = round(err, 5)
                    rec[f"{mode}_us"] = round(timeit(fn), 1)
                except Exception as exc:  # record unsupported modes
                    rec[f"{mode}_error"] = str(exc).splitlines()[0][:200]
            rec["bf16_us"] = round(timeit(lambda: torch.nn.functional.linear(x, w)), 1)
            out["results"].append(rec)
            print(json.dumps(rec), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "probe_fp8.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    sys.exit(main())
