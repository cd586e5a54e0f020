"""The register-fed 256x256 GEMM (csrc/kernels/gemm_w4r.hip) vs the fp32 PyTorch reference.  GPU only.

Shuffled-weight layout, every epilogue (store + bias, fused silu(gate)*up from the interleaved
copy, residual + bias), M and N not multiples of the tile (rows past M and a half panel past N
read zeros and are never stored: sentinel-checked), multi-item persistent streams and item
boundaries inside the prefetch window; asymmetric random data.
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


def _data(M, N, K, seed):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).to(torch.bfloat16)
    return x, w


def test_shuffle_layout(hip):
    """Element (panel p, k-block kb, n-block i, lane l, j) = W[64 p + 16 i + (l & 15)][32 kb + 8 (l >> 4) + j]."""
    N, K = 256, 128
    w = torch.arange(N * K, device="cuda", dtype=torch.float32).remainder(251).to(torch.bfloat16).view(N, K)
    s = hip.w4r_weight(w).view(N // 64, K // 32, 4, 64, 8)
    ref = w.view(N // 64, 4, 16, K // 32, 4, 8).permute(0, 3, 1, 4, 2, 5).reshape(N // 64, K // 32, 4, 64, 8)
    assert torch.equal(s, ref)
    # the SiLU copy: row 32 j + r of the interleaved view = gate 16 j + r (r < 16), up 16 j + r - 16
    I = N // 2
    inter = torch.cat([w[:I].view(I // 16, 16, K), w[I:].view(I // 16, 16, K)], dim=1).reshape(N, K)
    assert torch.equal(hip.w4r_weight(w, silu=True), hip.w4r_weight(inter.contiguous()))


@pytest.mark.parametrize("M,N,K", [(1, 256, 64), (300, 384, 256), (70, 320, 128), (1000, 1280, 320), (2500, 768, 1024),
                                   (4096, 5120, 5120)])
def test_w4r_store_bias(hip, M, N, K):
    x, w = _data(M, N, K, M + N)
    ws = hip.w4r_weight(w)
    b = torch.randn(N, device="cuda").to(torch.bfloat16)
    _close(hip.gemm_w4r(x, ws), _ref(x, w))
    _close(hip.gemm_w4r(x, ws, bias=b), _ref(x, w) + b.float())


@pytest.mark.parametrize("M,I,K", [(45, 256, 512), (700, 512, 256), (3000, 1024, 1024)])
def test_w4r_silu_mul(hip, M, I, K):
    x, w = _data(M, 2 * I, K, I + M)
    h = hip.gemm_w4r(x, hip.w4r_weight(w, silu=True), epi=1)
    gu = _ref(x, w)
    assert h.shape == (M, I)
    _close(h, torch.nn.functional.silu(gu[:, :I]) * gu[:, I:])


@pytest.mark.parametrize("M,N,K", [(333, 384, 128), (1500, 1024, 640), (4100, 2048, 2048)])
def test_w4r_residual(hip, M, N, K):
    x, w = _data(M, N, K, 7 * M + N)
    r = torch.randn(M, N, device="cuda").to(torch.bfloat16)
    b = torch.randn(N, device="cuda").to(torch.bfloat16)
    ref = r.float() + _ref(x, w)
    out = hip.gemm_w4r(x, hip.w4r_weight(w), epi=2, residual=r.clone(), out=torch.empty_like(r))
    _close(out, ref)
    rr = r.clone()
    hip.gemm_w4r(x, hip.w4r_weight(w), epi=2, residual=rr, out=rr, bias=b)  # in place (the engine's form)
    _close(rr, ref + b.float())


def test_w4r_rows_past_m_untouched(hip):
    """Output rows past M (a partial last m-tile) are never written: the output is a view into a
    larger sentinel-filled buffer."""
    M, N, K = 300, 384, 256
    x, w = _data(M, N, K, 5)
    buf = torch.full(((M + 64) * N,), 7.0, device="cuda", dtype=torch.bfloat16)
    y = hip.gemm_w4r(x, hip.w4r_weight(w), out=buf[:M * N].view(M, N))
    _close(y, _ref(x, w))
    assert torch.all(buf[M * N:] == 7.0)


def test_w4r_matches_w4(hip):
    """Same fp32 accumulation order per output element as the LDS-fed W4 kernel (cfg 11): bitwise."""
    M, N, K = 2048, 1024, 1024
    x, w = _data(M, N, K, 11)
    a = hip.gemm_w4r(x, hip.w4r_weight(w))
    b = hip.gemm_nt(x, w, 11, 0)
    assert torch.equal(a, b)
