"""Static ISA audit of the inline-asm MFMA GEMMs (gemm_w4.hip, gemm.hip, gemm_pp.hip) on the CPU.

Their MFMAs are inline asm, so hipcc neither pads their hazards nor sees their operands.
Three regressions this catches (each seen once while building the persistent four-wave kernel):

* a VALU write of an MFMA source register right before the asm MFMA (the zero-operand MFMAs
  that reset the accumulators between items read stale registers: every second item NaN);
* scratch in a W4 K-loop (an accumulator copy outside asm operands re-classed the
  accumulators and spilled ~300 registers); the split-K tails after the loop may spill a little;
* a counter wait other than the ring's own ``vmcnt(8)`` inside the W4 K-loop (an epilogue load
  left pending across the loop's back edge made hipcc put ``vmcnt(0)`` at the top of every
  K-tile, draining the LDS-DMA pieces in flight).
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
VALU_TO_MFMA_WAIT = 2  # wait states a VALU VGPR write needs before an MFMA reads it


def _compile(tmp_path_factory, name):
    if not shutil.which(HIPCC) and not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("isa") / f"{name}.s"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fgpu-flush-denormals-to-zero",
                    "-munsafe-fp-atomics", f"-I{ROOT}/csrc/kernels", "-S", "--cuda-device-only",
                    f"{ROOT}/csrc/kernels/{name}.hip", "-o", str(out)], check=True, capture_output=True)
    return out.read_text()


@pytest.fixture(scope="module", params=["gemm_w4", "gemm", "gemm_pp"])
def asm(request, tmp_path_factory):
    return request.param, _compile(tmp_path_factory, request.param)


def _kernels(text):
    return re.findall(r"^(_Z\S*):\s*; @\1\n(.*?)^\.Lfunc_end\d+:", text, re.M | re.S)


def _vregs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return {int(m.group(1))} if m else set()


def _hazards(body):
    """(VALU, MFMA) pairs where an inline-asm MFMA reads a VGPR a VALU op wrote < 2 wait states before."""
    lines = [ln.strip() for ln in body.split("\n")]
    out = []
    in_asm = False
    for i, ln in enumerate(lines):
        if ln.startswith(";;#ASMSTART"):
            in_asm = True
        elif ln.startswith(";;#ASMEND"):
            in_asm = False
        if not (in_asm and ln.startswith("v_mfma")):
            continue
        ops = [o.strip() for o in ln.split(None, 1)[1].split(",")]
        src = set().union(*(_vregs(o) for o in ops[1:4]))
        waits, k = 0, i - 1
        while k >= 0 and waits < VALU_TO_MFMA_WAIT:
            prev = lines[k]
            k -= 1
            if not prev or prev.startswith((";", ".")):
                if re.match(r"^\.LBB\d+_\d+:", prev):
                    break  # a block boundary: predecessors unknown, not judged
                continue
            if prev.startswith("v_") and not prev.startswith(("v_mfma", "v_accvgpr_read")):
                if _vregs(prev.split(None, 1)[1].split(",")[0].strip()) & src:
                    out.append((prev, ln))
            waits += int(prev.split()[1]) + 1 if prev.startswith("s_nop") else 1
    return out


def test_no_valu_write_right_before_asm_mfma(asm):
    name, text = asm
    bad = [(k, h) for k, body in _kernels(text) for h in _hazards(body)]
    assert not bad, (name, bad[:5])


def test_w4_kernels_spill_free_and_k_loop_waits_only_for_the_ring(asm):
    name, text = asm
    if name != "gemm_w4":
        pytest.skip("W4 only")
    kernels = [(k, b) for k, b in _kernels(text) if "gemm_w4_kernel" in k]
    assert len(kernels) == 5  # bf16 store / SiLU / residual, fp8 store / residual
    for k, body in kernels:
        lines = [ln.strip() for ln in body.split("\n")]
        blocks, cur = [], []
        for ln in lines:
            if re.match(r"^(\.LBB\d+_\d+:|; %bb\.\d+:)", ln):
                blocks.append(cur)
                cur = []
            cur.append(ln)
        blocks.append(cur)
        loop_blocks = [b for b in blocks if sum(x.startswith("v_mfma") for x in b) >= 16
                       and any("s_barrier" in x for x in b)]
        assert loop_blocks, k
        for b in loop_blocks:
            # the K-loop never touches scratch (the split-K / stream-K tails after it may: their
            # fp32 sums and epilogue share the register file with the 256 accumulators)
            assert not [x for x in b if x.startswith("scratch_")], k
            waits = [x for x in b if x.startswith("s_waitcnt") and "vmcnt" in x]
            assert all("vmcnt(8)" in x for x in waits), (k, waits)
        # and the tails' spill area stays small
        m = re.search(r"\.amdhsa_kernel " + re.escape(k) + r"\n.*?\.amdhsa_private_segment_fixed_size (\d+)",
                      text, re.S)
        assert m and int(m.group(1)) <= 2048, (k, m and m.group(1))
