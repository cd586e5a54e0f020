// FP8 (OCP e4m3fn, gfx950) activation quantisation for the fp8 projection path.
//
// Row-wise dynamic scaling: scale[r] = max|y[r,:]| / 448, q = y / scale
// (clamped to +-448, round-to-nearest-even by v_cvt_pk_fp8_f32).  The GEMM is
// hipBLASLt's fp8 kernel through torch._scaled_mm with row-wise scales on both
// operands (weights are quantised per output channel at load time), running at
// ~2x the bf16 rate.  The quantisation is fused into the producers so the fp8
// path adds no extra pass over the activations:
//   add_rmsnorm_fp8 : residual add + RMSNorm (bf16-rounded, as the bf16 path) + quant
//                     (also: plain RMSNorm + quant after a residual GEMM epilogue, and the
//                     embedding gather + RMSNorm + quant of the first layer)
//   silu_mul_fp8    : SiLU(gate) * up (bf16-rounded) + quant
//   quant_fp8       : stand-alone (attention output before o_proj)
// One 256-thread workgroup per row; the row max is a wave64 shuffle reduction
// plus 4 partials in LDS.

#include "common.h"

namespace {

constexpr int QT = 256;
constexpr float FP8_MAX = 448.f;
constexpr int NORM_MAX_CHUNK = 4;  // H <= 256 * 8 * 4

__device__ __forceinline__ uint32_t pack4_fp8(float a, float b, float c, float d) {
  const uint32_t lo = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  return __builtin_amdgcn_cvt_pk_fp8_f32(c, d, lo, true);
}

__device__ __forceinline__ float clampq(float v) { return fminf(fmaxf(v, -FP8_MAX), FP8_MAX); }

__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float m = red[0];
#pragma unroll
  for (int i = 1; i < QT / WAVE; ++i) m = fmaxf(m, red[i]);
  return m;
}

__device__ __forceinline__ float row_scale(float amax) { return fmaxf(amax, 1e-12f) / FP8_MAX; }

// store 8 quantised values (8 bytes)
__device__ __forceinline__ void store_q8(uint8_t* dst, const float (&y)[8], float scale) {
  uint2 p;
  p.x = pack4_fp8(clampq(y[0] / scale), clampq(y[1] / scale), clampq(y[2] / scale), clampq(y[3] / scale));
  p.y = pack4_fp8(clampq(y[4] / scale), clampq(y[5] / scale), clampq(y[6] / scale), clampq(y[7] / scale));
  *reinterpret_cast<uint2*>(dst) = p;
}

__global__ __launch_bounds__(QT) void quant_fp8_kernel(const bf16_t* __restrict__ x, uint8_t* __restrict__ q,
                                                       float* __restrict__ scale, int K) {
  __shared__ float red[QT / WAVE];
  const size_t base = static_cast<size_t>(blockIdx.x) * K;
  const int nvec = K / 8;
  float amax = 0.f;
  for (int vi = threadIdx.x; vi < nvec; vi += QT) {
    const u16x8 v = *reinterpret_cast<const u16x8*>(x + base + vi * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(bf2f(v[j])));
  }
  const float s = row_scale(block_max(amax, red));
  if (threadIdx.x == 0) scale[blockIdx.x] = s;
  for (int vi = threadIdx.x; vi < nvec; vi += QT) {
    const u16x8 v = *reinterpret_cast<const u16x8*>(x + base + vi * 8);
    float y[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) y[j] = bf2f(v[j]);
    store_q8(q + base + vi * 8, y, s);
  }
}

// has_residual: 0 = residual <- x, 1 = residual <- residual + x, 2 = plain RMSNorm of x (the
// residual stream was updated by the GEMM epilogue that produced x: nothing written back).
// gather != nullptr: x row = table row gather[row] (the embedding lookup fused in).
__global__ __launch_bounds__(QT) void add_rmsnorm_fp8_kernel(
    const bf16_t* __restrict__ x, bf16_t* __restrict__ residual, const bf16_t* __restrict__ w,
    uint8_t* __restrict__ q, float* __restrict__ scale, int H, float eps, int has_residual,
    const int* __restrict__ gather) {
  __shared__ float red[QT / WAVE];
  const int tid = threadIdx.x;
  const int nvec = H / 8;
  const size_t base = static_cast<size_t>(blockIdx.x) * H;
  // x row: the gathered table row (embedding lookup fused in) or this block's row
  const bf16_t* __restrict__ xr = gather ? x + static_cast<size_t>(gather[blockIdx.x]) * H : x + base;
  float v[NORM_MAX_CHUNK][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < NORM_MAX_CHUNK; ++c) {
    const int vi = tid + c * QT;
    if (vi < nvec) {
      const u16x8 xv = *reinterpret_cast<const u16x8*>(xr + vi * 8);
      u16x8 rv;
      if (has_residual == 1) rv = *reinterpret_cast<const u16x8*>(residual + base + vi * 8);
      u16x8 nr;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float f = bf2f(xv[j]);
        if (has_residual == 1) f += bf2f(rv[j]);
        nr[j] = f2bf(f);
        f = bf2f(nr[j]);
        v[c][j] = f;
        ss += f * f;
      }
      if (has_residual != 2) *reinterpret_cast<u16x8*>(residual + base + vi * 8) = nr;
    }
  }
  ss = wave_sum(ss);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int i = 0; i < QT / WAVE; ++i) tot += red[i];
  const float inv = rsqrtf(tot / H + eps);
  __syncthreads();  // red[] is reused by block_max
  float amax = 0.f;
#pragma unroll
  for (int c = 0; c < NORM_MAX_CHUNK; ++c) {
    const int vi = tid + c * QT;
    if (vi < nvec) {
      const u16x8 wv = *reinterpret_cast<const u16x8*>(w + vi * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[c][j] = bf2f(f2bf(v[c][j] * inv * bf2f(wv[j])));  // the bf16 path's rounding
        amax = fmaxf(amax, fabsf(v[c][j]));
      }
    }
  }
  const float s = row_scale(block_max(amax, red));
  if (tid == 0) scale[blockIdx.x] = s;
#pragma unroll
  for (int c = 0; c < NORM_MAX_CHUNK; ++c) {
    const int vi = tid + c * QT;
    if (vi < nvec) store_q8(q + base + vi * 8, v[c], s);
  }
}

__device__ __forceinline__ void silu8(const bf16_t* g, float (&y)[8], int I) {
  const u16x8 gv = *reinterpret_cast<const u16x8*>(g);
  const u16x8 uv = *reinterpret_cast<const u16x8*>(g + I);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float a = bf2f(gv[j]);
    y[j] = bf2f(f2bf(a / (1.f + __expf(-a)) * bf2f(uv[j])));
  }
}

__global__ __launch_bounds__(QT) void silu_mul_fp8_kernel(const bf16_t* __restrict__ gu, uint8_t* __restrict__ q,
                                                          float* __restrict__ scale, int I) {
  __shared__ float red[QT / WAVE];
  const bf16_t* row = gu + static_cast<size_t>(blockIdx.x) * 2 * I;
  uint8_t* qrow = q + static_cast<size_t>(blockIdx.x) * I;
  const int nvec = I / 8;
  float amax = 0.f;
  for (int vi = threadIdx.x; vi < nvec; vi += QT) {  // pass 1: row max (the row is re-read from L2 below)
    float y[8];
    silu8(row + vi * 8, y, I);
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(y[j]));
  }
  const float s = row_scale(block_max(amax, red));
  if (threadIdx.x == 0) scale[blockIdx.x] = s;
  for (int vi = threadIdx.x; vi < nvec; vi += QT) {
    float y[8];
    silu8(row + vi * 8, y, I);
    store_q8(qrow + vi * 8, y, s);
  }
}

}  // namespace

BCG_API int bcg_quant_fp8(const void* x, void* q, float* scale, int T, int K, hipStream_t stream) {
  if (K % 8 || T <= 0) return -2;
  hipLaunchKernelGGL(quant_fp8_kernel, dim3(T), dim3(QT), 0, stream, static_cast<const bf16_t*>(x),
                     static_cast<uint8_t*>(q), scale, K);
  return BCG_CHECK_LAUNCH();
}

BCG_API int bcg_add_rmsnorm_fp8(const void* x, void* residual, const void* w, void* q, float* scale, int T, int H,
                                float eps, int has_residual, hipStream_t stream) {
  if (H % 8 || H > QT * 8 * NORM_MAX_CHUNK || T <= 0 || has_residual < 0 || has_residual > 2) return -2;
  hipLaunchKernelGGL(add_rmsnorm_fp8_kernel, dim3(T), dim3(QT), 0, stream, static_cast<const bf16_t*>(x),
                     static_cast<bf16_t*>(residual), static_cast<const bf16_t*>(w), static_cast<uint8_t*>(q),
                     scale, H, eps, has_residual, static_cast<const int*>(nullptr));
  return BCG_CHECK_LAUNCH();
}

// residual[t] <- table[tokens[t]]; (q, scale)[t] <- fp8(rmsnorm(residual[t]) * w): the fp8 path's
// first layer input in one pass.  Token ids must be < vocab (checked by their producers).
BCG_API int bcg_embed_rmsnorm_fp8(const int* tokens, const void* table, const void* w, void* residual, void* q,
                                  float* scale, int T, int H, float eps, hipStream_t stream) {
  if (H % 8 || H > QT * 8 * NORM_MAX_CHUNK || T <= 0) return -2;
  hipLaunchKernelGGL(add_rmsnorm_fp8_kernel, dim3(T), dim3(QT), 0, stream, static_cast<const bf16_t*>(table),
                     static_cast<bf16_t*>(residual), static_cast<const bf16_t*>(w), static_cast<uint8_t*>(q),
                     scale, H, eps, 0, tokens);
  return BCG_CHECK_LAUNCH();
}

BCG_API int bcg_silu_mul_fp8(const void* gu, void* q, float* scale, int T, int I, hipStream_t stream) {
  if (I % 8 || T <= 0) return -2;
  hipLaunchKernelGGL(silu_mul_fp8_kernel, dim3(T), dim3(QT), 0, stream, static_cast<const bf16_t*>(gu),
                     static_cast<uint8_t*>(q), scale, I);
  return BCG_CHECK_LAUNCH();
}
