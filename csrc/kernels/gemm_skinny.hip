// Decode-shaped GEMM on MFMA: y[M,N] = x[M,K] · W[N,K]^T (+ bias), M <= 192.
//
// Decode projections are weight-streaming problems (every weight byte is used
// M times, M = number of live sequences): the kernel is built to keep HBM busy,
// not the matrix cores.
//   * one wave owns 32 output features (two 16-wide n-tiles) for ALL M rows
//     (MT 16-row m-tiles); a 256-thread workgroup covers 128 features;
//   * both operands are loaded straight into MFMA fragments with 16-byte
//     loads (guide: "GEMV / M <= 16 ... load straight to VGPRs, deep unroll"):
//       W (B operand): lane l -> W[n0 + (l&15)][k0 + 8(l>>4) .. +8]
//       x (A operand): lane l -> x[m0 + (l&15)][k0 + 8(l>>4) .. +8]   (L1/L2 resident)
//     four 32-deep k-steps are issued before the first MFMA that needs them;
//   * split-K over workgroups when N/128 alone cannot fill 256 CUs; partial
//     sums go through fp32 atomics into a zeroed workspace and a small
//     epilogue kernel converts (+bias) to bf16.
// x (<= 128 x K bf16, <= 4.5 MB) is re-read by every workgroup from L2; W is
// streamed exactly once, so no XCD-aware placement is needed here.

#include "common.h"

namespace {

// U = k-steps (of 32) issued ahead: 4 for small M, 2 when the x fragments of
// many m-tiles would not fit the register file.
template <int MT, int U>
__global__ __launch_bounds__(256) void gemm_skinny_kernel(const bf16_t* __restrict__ x,
                                                          const bf16_t* __restrict__ w,
                                                          const bf16_t* __restrict__ bias,
                                                          bf16_t* __restrict__ y, float* __restrict__ ws,
                                                          int M, int N, int K, int split_k, int ksteps_per) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r = lane & 15, h = lane >> 4;
  const int nblocks = N / 128;
  const int nb = blockIdx.x % nblocks;
  const int ks = blockIdx.x / nblocks;
  const int n0 = nb * 128 + wave * 32;
  const int kstep0 = ks * ksteps_per;
  const int kstep1 = min(K / 32, kstep0 + ksteps_per);

  f32x4 acc[MT][2];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    acc[mt][0] = f32x4{0.f, 0.f, 0.f, 0.f};
    acc[mt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const bf16_t* w0 = w + static_cast<size_t>(n0 + r) * K + 8 * h;
  const bf16_t* w1 = w0 + static_cast<size_t>(16) * K;
  const bf16_t* xr[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) xr[mt] = x + static_cast<size_t>(min(mt * 16 + r, M - 1)) * K + 8 * h;

  for (int kst = kstep0; kst < kstep1; kst += U) {
    bf16x8 bw0[U], bw1[U], ax[U][MT];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = (kst + u) * 32;
      bw0[u] = *reinterpret_cast<const bf16x8*>(w0 + k);
      bw1[u] = *reinterpret_cast<const bf16x8*>(w1 + k);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int k = (kst + u) * 32;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) ax[u][mt] = *reinterpret_cast<const bf16x8*>(xr[mt] + k);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        acc[mt][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ax[u][mt], bw0[u], acc[mt][0], 0, 0, 0);
        acc[mt][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ax[u][mt], bw1[u], acc[mt][1], 0, 0, 0);
      }
  }

  // C layout: lane holds rows m = mt*16 + 4h + i, column n = n0 + nt*16 + r
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int n = n0 + nt * 16 + r;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = mt * 16 + 4 * h + i;
        if (m >= M) continue;
        const float v = acc[mt][nt][i];
        if (split_k == 1) {
          const float b = bias ? bf2f(bias[n]) : 0.f;
          y[static_cast<size_t>(m) * N + n] = f2bf(v + b);
        } else {
          atomicAdd(ws + static_cast<size_t>(m) * N + n, v);
        }
      }
    }
}

__global__ __launch_bounds__(256) void splitk_epilogue_kernel(const float* __restrict__ ws,
                                                              const bf16_t* __restrict__ bias,
                                                              bf16_t* __restrict__ y, int M, int N) {
  const int64_t total = static_cast<int64_t>(M) * N / 4;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(blockDim.x) + threadIdx.x; i < total;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const f32x4 v = reinterpret_cast<const f32x4*>(ws)[i];
    const int n = static_cast<int>((i * 4) % N);
    u16x4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = f2bf(v[j] + (bias ? bf2f(bias[n + j]) : 0.f));
    reinterpret_cast<u16x4*>(y)[i] = o;
  }
}

template <int MT>
void launch(const bf16_t* x, const bf16_t* w, const bf16_t* bias, bf16_t* y, float* ws, int M, int N, int K,
            int split_k, hipStream_t s) {
  constexpr int U = MT <= 4 ? 4 : 2;
  const int ksteps = K / 32;
  const int per = ((ksteps + split_k - 1) / split_k + U - 1) / U * U;
  const int splits = (ksteps + per - 1) / per;  // no workgroup without k-steps
  const int grid = (N / 128) * splits;
  hipLaunchKernelGGL((gemm_skinny_kernel<MT, U>), dim3(grid), dim3(256), 0, s, x, w, bias, y, ws, M, N, K, split_k, per);
}

}  // namespace

// Host picks split_k (1 = no workspace needed); ws must hold M*N floats, zeroed, when split_k > 1.
BCG_API int bcg_gemm_skinny(const void* x, const void* w, const void* bias, void* y, float* ws, int M, int N,
                            int K, int split_k, hipStream_t stream) {
  if (M <= 0 || M > 192 || N % 128 || K % 128 || split_k < 1) return -2;
  if (split_k > 1 && ws == nullptr) return -2;
  const bf16_t* xb = static_cast<const bf16_t*>(x);
  const bf16_t* wb = static_cast<const bf16_t*>(w);
  const bf16_t* bb = static_cast<const bf16_t*>(bias);
  bf16_t* yb = static_cast<bf16_t*>(y);
  const int MT = (M + 15) / 16;
  switch (MT) {
    case 1: launch<1>(xb, wb, bb, yb, ws, M, N, K, split_k, stream); break;
    case 2: launch<2>(xb, wb, bb, yb, ws, M, N, K, split_k, stream); break;
    case 3: launch<3>(xb, wb, bb, yb, ws, M, N, K, split_k, stream); break;
    case 4: launch<4>(xb, wb, bb, yb, ws, M, N, K, split_k, stream); break;
    case 5: launch<5>(xb, wb, bb, yb, ws, M, N, K, split_k, stream); break;
    case 6: launch<6>(xb, wb, bb, yb, ws, M, N, K, split_k, stream); break;
    case 7: launch<7>(xb, wb, bb, yb, ws, M, N, K, split_k, stream); break;
    case 8: launch<8>(xb, wb, bb, yb, ws, M, N, K, split_k, stream); break;
    case 9: launch<9>(xb, wb, bb, yb, ws, M, N, K, split_k, stream); break;
    case 10: launch<10>(xb, wb, bb, yb, ws, M, N, K, split_k, stream); break;
    case 11: launch<11>(xb, wb, bb, yb, ws, M, N, K, split_k, stream); break;
    default: launch<12>(xb, wb, bb, yb, ws, M, N, K, split_k, stream); break;
  }
  if (split_k > 1) {
    const int64_t work = static_cast<int64_t>(M) * N / 4;
    const int blocks = static_cast<int>(std::min<int64_t>((work + 255) / 256, 2048));
    hipLaunchKernelGGL(splitk_epilogue_kernel, dim3(blocks), dim3(256), 0, stream, ws, bb, yb, M, N);
  }
  return BCG_CHECK_LAUNCH();
}
