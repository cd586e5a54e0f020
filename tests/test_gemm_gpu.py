"""Hand MFMA GEMM (csrc/kernels/gemm.hip) vs the fp32 PyTorch reference.  GPU only.

Every tile configuration and epilogue (store + bias, fused silu(gate)*up,
fused residual add) on decode-shaped problems, M not a multiple of the tile,
with asymmetric random data (a row/column swap of the output or a gate/up
mix-up cannot pass).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hip():
    from byzantine_consensus_llm_agents_amd.ops import get_ops
    return get_ops("hip")


def _ref(x, w):
    return x.float() @ w.float().t()


def _close(a, b, tol=2e-2):
    err = (a.float() - b.float()).abs().max().item()
    scale = b.float().abs().max().item()
    assert err <= tol * max(1.0, scale), (err, scale)


@pytest.mark.parametrize("cfg", list(range(12)))
@pytest.mark.parametrize("M,N,K", [(37, 256, 512), (200, 768, 1024), (448, 1280, 5120), (1, 256, 128)])
def test_gemm_store_bias(hip, cfg, M, N, K):
    torch.manual_seed(M + N + cfg)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    b = torch.randn(N, device="cuda").to(torch.bfloat16)
    if not hip.gemm_plan.supported(cfg, M, N, K, 0):
        pytest.skip("shape not a multiple of this tile")
    y = hip.gemm_nt(x, w, cfg, 0)
    _close(y, _ref(x, w))
    yb = hip.gemm_nt(x, w, cfg, 0, bias=b)
    _close(yb, _ref(x, w) + b.float())


@pytest.mark.parametrize("cfg", list(range(12)))
@pytest.mark.parametrize("M,I,K", [(45, 256, 512), (300, 1024, 1024)])
def test_gemm_silu_mul_epilogue(hip, cfg, M, I, K):
    torch.manual_seed(I + cfg)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(2 * I, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    if not hip.gemm_plan.supported(cfg, M, 2 * I, K, 1):
        pytest.skip("shape not a multiple of this tile")
    h = hip.gemm_nt(x, w, cfg, 1)
    gu = _ref(x, w)
    ref = torch.nn.functional.silu(gu[:, :I]) * gu[:, I:]
    assert h.shape == (M, I)
    _close(h, ref)


@pytest.mark.parametrize("cfg", [0, 1, 3, 10, 11])
def test_gemm_residual_epilogue_in_place(hip, cfg):
    torch.manual_seed(cfg)
    M, N, K = 77, 512, 2048
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    r = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    ref = r.float() + _ref(x, w)
    out = hip.gemm_nt(x, w, cfg, 2, residual=r, out=r)  # in place, as the model uses it
    assert out.data_ptr() == r.data_ptr()
    _close(r, ref)


@pytest.mark.parametrize("cfg,split", [(0, 2), (5, 3), (6, 4), (2, 8), (1, 6), (7, 2), (9, 3), (10, 2), (10, 3),
                                       (10, 5), (11, 2), (11, 3), (11, 5)])
@pytest.mark.parametrize("epi", [0, 1, 2])
def test_gemm_split_k(hip, cfg, split, epi):
    """Split-K with the in-kernel last-arriver reduction, repeated launches (the counters
    must be left zeroed for the next launch, as inside a replayed graph)."""
    torch.manual_seed(split + epi)
    M, N, K = 150, 1024, 4096
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    ref = _ref(x, w)
    if epi == 1:
        ref = torch.nn.functional.silu(ref[:, :N // 2]) * ref[:, N // 2:]
    for _ in range(3):
        if epi == 2:
            r = torch.randn(M, N, device="cuda").to(torch.bfloat16)
            want = r.float() + ref
            got = hip.gemm_nt(x, w, cfg, 2, residual=r, out=r, split_k=split)
        else:
            want = ref
            got = hip.gemm_nt(x, w, cfg, epi, split_k=split)
        _close(got, want)


def test_fused_ops_match_unfused(hip):
    """linear_silu / linear_residual (whatever path the plan picks) == the unfused ops."""
    torch.manual_seed(1)
    M, H, I = 96, 1024, 1536
    x = torch.randn(M, H, device="cuda").to(torch.bfloat16)
    wgu = (torch.randn(2 * I, H, device="cuda") * H ** -0.5).to(torch.bfloat16)
    wd = (torch.randn(H, I, device="cuda") * I ** -0.5).to(torch.bfloat16)
    r = torch.randn(M, H, device="cuda").to(torch.bfloat16)
    h = hip.linear_silu(x, wgu)
    _close(h, hip.silu_mul(torch.nn.functional.linear(x, wgu)), 3e-2)
    ref = r.float() + _ref(h, wd)
    _close(hip.linear_residual(h, wd, r.clone()), ref, 3e-2)


@pytest.mark.parametrize("M,N,K", [(300, 1040, 64), (257, 528, 128), (513, 784, 192), (1, 4112, 320),
                                   (768, 2048, 1024)])
@pytest.mark.parametrize("epi", [0, 2])
@pytest.mark.parametrize("cfg", [10, 11])
def test_gemm_pp_edges(hip, M, N, K, epi, cfg):
    """The 256x256 kernels (cfg 10 ping-pong, cfg 11 four-wave) at their edges: 1-3
    K-tiles (prologue-only pipelines), M and N not multiples of the tile (clamped / range-checked
    loads, masked stores: the LM head has N = 151936 = 593.5 tiles), repeated launches."""
    torch.manual_seed(M * 7 + N + K)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    ref = _ref(x, w)
    for _ in range(2):
        if epi == 2:
            r = torch.randn(M, N, device="cuda").to(torch.bfloat16)
            want = r.float() + ref
            got = hip.gemm_nt(x, w, cfg, 2, residual=r, out=r)
        else:
            want = ref
            got = hip.gemm_nt(x, w, cfg, 0)
        _close(got, want)


@pytest.mark.parametrize("cfg", [10, 11])
@pytest.mark.parametrize("M,N,K", [(77, 528, 1024), (1500, 4112, 512)])
def test_gemm_residual_plus_bias(hip, cfg, M, N, K):
    """The 256x256 kernels' residual epilogue with a bias as well (both added in fp32), partial
    tiles in M and N, bf16 and fp8."""
    torch.manual_seed(M + N + cfg)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    b = torch.randn(N, device="cuda").to(torch.bfloat16)
    r = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    want = r.float() + b.float() + _ref(x, w)
    _close(hip.gemm_nt(x, w, cfg, 2, bias=b, residual=r, out=r), want)
    xq, xs, wq, ws, ref = _fp8_operands(M, N, K, 3 + cfg)
    r = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    want = r.float() + b.float() + ref
    _close(hip.gemm_nt_fp8(xq, xs, wq, ws, cfg, 2, bias=b, residual=r, out=r), want)


@pytest.mark.parametrize("M,N,K", [(4096 + 77, 4112, 1024), (16384, 1280, 256), (9000, 2560, 64), (300, 74752, 128)])
@pytest.mark.parametrize("epi", [0, 1, 2])
def test_gemm_w4_persistent_many_items(hip, M, N, K, epi):
    """cfg 11's persistent launch: more tiles than CUs, so a workgroup streams several items
    (epilogue of one while the next one's first K-tiles land), partial last tiles in M and N,
    1-16 K-tiles per item, repeated launches."""
    torch.manual_seed(M + N + K + epi)
    if epi == 1:
        N -= N % 256  # (the fused SiLU needs inter % 128 == 0)
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    ref = _ref(x, w)
    for _ in range(2):
        if epi == 2:
            r = torch.randn(M, N, device="cuda").to(torch.bfloat16)
            want = r.float() + ref
            _close(hip.gemm_nt(x, w, 11, 2, residual=r, out=r), want)
        elif epi == 1:
            I = N // 2
            _close(hip.gemm_nt(x, w, 11, 1), torch.nn.functional.silu(ref[:, :I]) * ref[:, I:])
        else:
            _close(hip.gemm_nt(x, w, 11, 0), ref)


@pytest.mark.parametrize("cfg", [10, 11])
def test_gemm_pp_prefill_chunk_silu(hip, cfg):
    """A prefill-sized gate_up chunk through the 256x256 kernels with the fused SiLU*mul."""
    torch.manual_seed(5)
    M, I, K = 2048 + 77, 1408, 2048
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(2 * I, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    gu = _ref(x, w)
    ref = torch.nn.functional.silu(gu[:, :I]) * gu[:, I:]
    _close(hip.gemm_nt(x, w, cfg, 1), ref)


# ---- fp8 (e4m3fn) variant: xs[m] * ws[n] * (xq . wq^T), block-scaled K = 128 MFMA ----------
def _fp8_operands(M, N, K, seed):
    from byzantine_consensus_llm_agents_amd.ops.reference import quant_fp8
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).to(torch.bfloat16)
    xq, xs = quant_fp8(x)
    wq, ws = quant_fp8(w)
    ref = (xq.float() * xs[:, None]) @ (wq.float() * ws[:, None]).t()  # exact dequantised operands
    return xq, xs, wq, ws, ref


@pytest.mark.parametrize("cfg", list(range(12)))
@pytest.mark.parametrize("M,N,K", [(37, 256, 512), (200, 768, 1024), (448, 1280, 6144), (1, 256, 128)])
def test_gemm_fp8_store_bias(hip, cfg, M, N, K):
    bm, bn = hip.gemm_plan.tiles[cfg]
    if N % bn:
        pytest.skip("N not a multiple of this tile")
    xq, xs, wq, ws, ref = _fp8_operands(M, N, K, M + N + cfg)
    b = torch.randn(N, device="cuda").to(torch.bfloat16)
    _close(hip.gemm_nt_fp8(xq, xs, wq, ws, cfg), ref)
    _close(hip.gemm_nt_fp8(xq, xs, wq, ws, cfg, bias=b), ref + b.float())


@pytest.mark.parametrize("cfg,split", [(0, 2), (9, 3), (1, 4)])
def test_gemm_fp8_split_k_residual(hip, cfg, split):
    M, N, K = 300, 1024, 2048
    xq, xs, wq, ws, ref = _fp8_operands(M, N, K, 7 + cfg)
    r = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    want = ref + r.float()
    y = hip.gemm_nt_fp8(xq, xs, wq, ws, (cfg, split), 2, residual=r.clone())
    _close(y, want)
    for _ in range(2):  # counters left zeroed: repeated launches stay correct
        _close(hip.gemm_nt_fp8(xq, xs, wq, ws, (cfg, split)), ref)


def test_linear_fp8_dispatch_matches_library(hip):
    """The decode-size fp8 projection goes to the hand kernel and matches hipBLASLt's _scaled_mm."""
    M, N, K = 160, 8192, 6144  # Mistral-Small-22B qkv at a decode bucket
    xq, xs, wq, ws, ref = _fp8_operands(M, N, K, 11)
    assert hip.fp8_cfg(M, N, K) is not None
    y = hip.linear_fp8(xq, xs, wq, ws)
    lib = torch._scaled_mm(xq, wq.t(), scale_a=xs.view(-1, 1), scale_b=ws.view(1, -1), out_dtype=torch.bfloat16)
    _close(y, ref)
    _close(y, lib.float())


@pytest.mark.parametrize("M,N,K,split", [(300, 1040, 128, 1), (2048 + 77, 1536, 1024, 1), (1, 4112, 384, 1),
                                         (513, 784, 1024, 3), (4096, 6144, 2048, 1)])
@pytest.mark.parametrize("epi", [0, 2])
@pytest.mark.parametrize("cfg", [10, 11])
def test_gemm_pp_fp8(hip, M, N, K, split, epi, cfg):
    """The 256x256 kernels' fp8 forms (cfg 10 ping-pong: 16x16x128 block-scaled MFMAs; cfg 11
    four-wave: 32x32x64): edges (1-3 K-tiles, partial tiles in M and N), split-K, residual
    epilogue, repeated launches."""
    xq, xs, wq, ws, ref = _fp8_operands(M, N, K, M + N + K + epi)
    b = torch.randn(N, device="cuda").to(torch.bfloat16)
    for _ in range(2):
        if epi == 2:
            r = torch.randn(M, N, device="cuda").to(torch.bfloat16)
            want = ref + r.float() + b.float()
            got = hip.gemm_nt_fp8(xq, xs, wq, ws, (cfg, split), 2, bias=b, residual=r, out=r)
        else:
            want = ref + b.float()
            got = hip.gemm_nt_fp8(xq, xs, wq, ws, (cfg, split), 0, bias=b)
        _close(got, want)


@pytest.mark.parametrize("cfg", [10, 11])
@pytest.mark.parametrize("epi", [0, 1, 2])
@pytest.mark.parametrize("M", [37, 257])
def test_gemm_big_tile_partial_m_leaves_rows_past_m(hip, cfg, epi, M):
    """A partial last M tile of the 256x256 kernels must not touch rows >= M: the output (and
    residual) are views buf[:M] of a larger buffer whose extra rows hold a sentinel."""
    torch.manual_seed(M + epi)
    N, K = 512, 1024
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    width = N // 2 if epi == 1 else N
    buf = torch.full((M + 256, width), 7.0, device="cuda", dtype=torch.bfloat16)
    out = buf[:M]
    ref = _ref(x, w)
    if epi == 1:
        ref = torch.nn.functional.silu(ref[:, :width]) * ref[:, width:]
    res = None
    if epi == 2:
        rbuf = torch.full((M + 256, N), -3.0, device="cuda", dtype=torch.bfloat16)
        rbuf[:M] = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        res = rbuf[:M]
        ref = ref + res.float()
    got = hip.gemm_nt(x, w, cfg, epi, residual=res, out=out)
    _close(got, ref)
    assert torch.all(buf[M:] == 7.0), "rows past M were written"
    if epi == 2:
        assert torch.all(rbuf[M:] == -3.0)


@pytest.mark.parametrize("cfg", [10, 11])
@pytest.mark.parametrize("epi", [0, 2])
@pytest.mark.parametrize("M", [37, 257])
def test_gemm_fp8_big_tile_partial_m_leaves_rows_past_m(hip, cfg, epi, M):
    N, K = 512, 1024
    xq, xs, wq, ws, ref = _fp8_operands(M, N, K, 3 * M + epi)
    buf = torch.full((M + 256, N), 7.0, device="cuda", dtype=torch.bfloat16)
    res = None
    if epi == 2:
        res = torch.randn(M, N, device="cuda").to(torch.bfloat16)
        buf[:M] = res
        ref = ref + res.float()
        res = buf[:M]
    got = hip.gemm_nt_fp8(xq, xs, wq, ws, cfg, epi, residual=res, out=buf[:M])
    _close(got, ref)
    assert torch.all(buf[M:] == 7.0), "rows past M were written"


@pytest.mark.parametrize("M,N,K", [(37, 512, 1024), (704, 1040, 5120), (257, 34816 // 8, 640), (2048 + 77, 1536, 2048),
                                   (704, 7168, 5120), (1, 256, 128)])
@pytest.mark.parametrize("epi", [0, 1, 2])
def test_gemm_w4_stream_k(hip, M, N, K, epi):
    """W4 stream-K (split_k = 0): one workgroup per CU over the tiles x K-tiles units, partial
    tiles summed by the last-arriving wave after its stream.  Store + bias, SiLU, residual in
    place (bias too); rows past M untouched; repeated launches (counters left zeroed)."""
    torch.manual_seed(M + N + epi)
    if epi == 1 and (N // 2) % 128:
        pytest.skip("silu: inter % 128")
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
    b = torch.randn(N, device="cuda").to(torch.bfloat16)
    assert hip.gemm_plan.supported(11, M, N, K, epi, 0)
    ref = _ref(x, w)
    width = N // 2 if epi == 1 else N
    for rep in range(3):
        buf = torch.full((M + 256, width), 7.0, device="cuda", dtype=torch.bfloat16)
        if epi == 0:
            got = hip.gemm_nt(x, w, (11, 0), 0, bias=b, out=buf[:M])
            want = ref + b.float()
        elif epi == 1:
            got = hip.gemm_nt(x, w, (11, 0), 1, out=buf[:M])
            want = torch.nn.functional.silu(ref[:, :width]) * ref[:, width:]
        else:
            buf[:M] = torch.randn(M, N, device="cuda").to(torch.bfloat16)
            want = ref + buf[:M].float() + b.float()
            got = hip.gemm_nt(x, w, (11, 0), 2, bias=b, residual=buf[:M], out=buf[:M])
        _close(got, want)
        assert torch.all(buf[M:] == 7.0), "rows past M were written"
