"""Static audit of the register-staged 256x256 GEMM (csrc/experimental/gemm_rs.hip) on the CPU host.

Its MFMAs are inline asm with AGPR-pinned accumulators, so hipcc pads no MFMA hazard for
them and would not notice if an accumulator were spilled: an MFMA result copied or stored
right after the instruction reads the OLD value (seen once: a rolled schedule loop put the
accumulators in scratch and every output came back zero).  This test compiles the kernel
for gfx950 (hipcc cross-compiles without a GPU) and checks the emitted main loop: 128 MFMAs
on 64 distinct accumulator blocks, no scratch access and no compiler AGPR move inside it,
and nothing touching the accumulators between the loop exit and the hazard padding.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    if not shutil.which(HIPCC) and not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("isa") / "gemm_rs.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fgpu-flush-denormals-to-zero",
                    "-munsafe-fp-atomics", f"-I{ROOT}/csrc/kernels", "-S", "--cuda-device-only",
                    f"{ROOT}/csrc/experimental/gemm_rs.hip", "-o", str(out)], check=True, capture_output=True)
    return out.read_text()


def _kernels(text):
    return re.findall(r"^(_Z\S*gemm_rs_kernel\S*):\s*; @\1\n(.*?)^\.Lfunc_end\d+:", text, re.M | re.S)


def test_gemm_rs_main_loop_is_clean(asm):
    kernels = _kernels(asm)
    assert len(kernels) == 3  # the three epilogues
    for name, body in kernels:
        lines = [l.strip() for l in body.split("\n")]
        labels = {l.split(":")[0]: i for i, l in enumerate(lines) if re.match(r"^\.LBB\d+_\d+:", l)}
        loops = []
        for i, l in enumerate(lines):
            m = re.match(r"^s_cbranch_\w+\s+(\.LBB\d+_\d+)", l)
            if m and labels.get(m.group(1), i) < i:
                loops.append((labels[m.group(1)], i))
        mfma_loops = [(a, b) for a, b in loops if any(x.startswith("v_mfma") for x in lines[a:b])]
        assert len(mfma_loops) == 1, (name, mfma_loops)
        a, b = mfma_loops[0]
        seg = lines[a:b + 1]
        mfma = [x for x in seg if x.startswith("v_mfma")]
        assert len(mfma) == 128, (name, len(mfma))
        dsts = {re.match(r"v_mfma\S+\s+(a\[\d+:\d+\])", x).group(1) for x in mfma}
        assert len(dsts) == 64, (name, len(dsts))
        assert not [x for x in seg if x.startswith("scratch_")], name
        assert not [x for x in seg if x.startswith("v_accvgpr")], name
        # between the loop exit and the padding: no accumulator reader
        nop = next(i for i in range(b, len(lines)) if lines[i].startswith("s_nop 7"))
        for x in lines[b + 1:nop]:
            assert not (x.startswith(("scratch_", "v_accvgpr_read", "global_store", "buffer_store"))
                        or re.search(r"\ba\[\d+", x)), (name, x)
