"""Profiling tools on synthetic rocprofv3 traces (CPU): the prefill / decode split of
tools/phase_split.py that PERF.md's steady-state breakdown comes from."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _trace(path):
    rows, t = [], 0

    def k(name, dur):
        nonlocal t
        rows.append({"Kernel_Name": name, "Start_Timestamp": t, "End_Timestamp": t + dur, "Queue_Id": 1})
        t += dur + 1

    for _ in range(2):  # a 2-layer prefill forward
        for name in ("add_rmsnorm_kernel", "Cijk_qkv", "qk_norm_rope_kv_vec_kernel", "prefill_attn_kernel<128>",
                     "gemm_pp_kernel<2>", "add_rmsnorm_kernel", "gemm_pp_kernel<1>", "Cijk_down_SK3"):
            k(name, 100)
    for _ in range(3):  # 3 decode steps of the same model
        for _ in range(2):
            for name in ("add_rmsnorm_kernel", "gemm_nt_kernel", "qk_norm_rope_kv_vec_kernel", "decode_shared_kernel",
                         "decode_attn_kernel<128>", "decode_combine_kernel", "gemm_nt_kernel", "add_rmsnorm_kernel",
                         "gemm_pp_kernel<1>", "gemm_nt_kernel"):
                k(name, 10)
        k("guided_sample_kernel", 5)
    with open(path, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=list(rows[0]))
        w.writeheader()
        w.writerows(rows)


def test_phase_split_assigns_kernels_to_their_forward(tmp_path):
    path = str(tmp_path / "trace.csv")
    _trace(path)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "phase_split.py"), path],
                         stdout=subprocess.PIPE, check=True, text=True).stdout
    d = json.loads(out)
    pre, dec = d["prefill"]["families_ms"], d["decode"]["families_ms"]
    # 16 prefill kernels x 100 ns against 3 x (2 x 10 x 10 + 5) ns of decode: the decode layers'
    # input norm at the switch belongs to decode, the prefill tail (o / gate_up / down) to prefill
    assert abs(d["prefill"]["share_of_kernel_time"] - 1600 / 2215) < 1e-3
    assert abs(d["decode"]["share_of_kernel_time"] - 615 / 2215) < 1e-3
    assert set(pre) == {"norm", "gemm_hipblaslt", "rope_kv", "attn_prefill", "gemm_hand_256x256"}
    assert {"attn_decode", "attn_decode_shared", "attn_decode_combine", "sampler"} <= set(dec)
