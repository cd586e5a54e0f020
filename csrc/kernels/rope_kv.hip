// Fused QKV epilogue: split -> (Qwen3) per-head RMSNorm -> neox RoPE -> paged KV write.
//
// One wave64 per (token, head-slot); slots [0,n_q) are query heads (written
// to q_out[T,n_q,hd]), [n_q,n_q+n_kv) key heads, the rest value heads.  Lane
// l owns the rotation pair (l, l+hd/2) so RoPE needs no cross-lane traffic;
// the head RMS is one wave reduction.  cos/sin come from a precomputed fp32
// table [max_pos, hd] (first half cos, second half sin) -- no on-device trig.
//
// KV cache layouts (see ops/reference.py):
//   K: [L, NB, n_kv, BS, hd]   (token rows: the A operand of S^T = K Q^T)
//   V: [L, NB, n_kv, hd, BS]   (transposed: the A operand of O^T = V^T P^T)
// Element type: bf16, or OCP fp8 e4m3fn (kv_fp8; scale 1, saturated to
// +-448, round-to-nearest-even) -- half the KV bytes every decode step streams.

#include "common.h"

namespace {

constexpr int HEADS_PER_BLOCK = 4;  // 4 waves per 256-thread workgroup

template <typename T>
__device__ __forceinline__ T to_cache(float f);
template <>
__device__ __forceinline__ bf16_t to_cache<bf16_t>(float f) { return f2bf(f); }
template <>
__device__ __forceinline__ uint8_t to_cache<uint8_t>(float f) {
  f = fminf(fmaxf(f, -448.f), 448.f);  // e4m3fn has no inf: saturate
  return static_cast<uint8_t>(__builtin_amdgcn_cvt_pk_fp8_f32(f, 0.f, 0, false) & 0xff);
}

template <typename CacheT>
__global__ __launch_bounds__(256) void qk_norm_rope_kv_kernel(
    const bf16_t* __restrict__ qkv, const int* __restrict__ positions, const int* __restrict__ slots,
    bf16_t* __restrict__ q_out, const bf16_t* __restrict__ q_norm, const bf16_t* __restrict__ k_norm,
    const float* __restrict__ cos_sin, CacheT* __restrict__ k_cache, CacheT* __restrict__ v_cache,
    int layer, int T, int n_q, int n_kv, int hd, int num_blocks, int block_size, float eps) {
  const int lane = threadIdx.x & 63;
  const int slot_head = blockIdx.y * HEADS_PER_BLOCK + (threadIdx.x >> 6);
  const int t = blockIdx.x;
  const int n_heads = n_q + 2 * n_kv;
  if (slot_head >= n_heads || t >= T) return;
  const int half = hd >> 1;
  const bool active = lane < half;
  const size_t row = static_cast<size_t>(t) * n_heads * hd;
  const bf16_t* src = qkv + row + static_cast<size_t>(slot_head) * hd;
  float x1 = active ? bf2f(src[lane]) : 0.f;
  float x2 = active ? bf2f(src[lane + half]) : 0.f;

  const int slot = slots[t];
  const int blk = slot / block_size, off = slot % block_size;

  if (slot_head >= n_q + n_kv) {  // value head: transposed store, no transform
    const int h = slot_head - n_q - n_kv;
    const size_t vbase = ((static_cast<size_t>(layer) * num_blocks + blk) * n_kv + h) * hd * block_size;
    if (active) {
      v_cache[vbase + static_cast<size_t>(lane) * block_size + off] = to_cache<CacheT>(x1);
      v_cache[vbase + static_cast<size_t>(lane + half) * block_size + off] = to_cache<CacheT>(x2);
    }
    return;
  }
  const bool is_q = slot_head < n_q;
  const bf16_t* nw = is_q ? q_norm : k_norm;
  if (nw != nullptr) {
    const float ss = wave_sum(x1 * x1 + x2 * x2);
    const float inv = rsqrtf(ss / hd + eps);
    if (active) {
      x1 = x1 * inv * bf2f(nw[lane]);
      x2 = x2 * inv * bf2f(nw[lane + half]);
    }
  }
  if (!active) return;
  const float* cs = cos_sin + static_cast<size_t>(positions[t]) * hd;
  const float c = cs[lane], s = cs[half + lane];
  const float y1 = x1 * c - x2 * s;
  const float y2 = x2 * c + x1 * s;
  if (is_q) {
    bf16_t* dst = q_out + (static_cast<size_t>(t) * n_q + slot_head) * hd;
    dst[lane] = f2bf(y1);
    dst[lane + half] = f2bf(y2);
  } else {
    const int h = slot_head - n_q;
    CacheT* dst = k_cache + (((static_cast<size_t>(layer) * num_blocks + blk) * n_kv + h) * block_size + off) * hd;
    dst[lane] = to_cache<CacheT>(y1);
    dst[lane + half] = to_cache<CacheT>(y2);
  }
}

}  // namespace

BCG_API int bcg_qk_norm_rope_kv_write(const void* qkv, const int* positions, const int* slots, void* q_out,
                                      const void* q_norm, const void* k_norm, const float* cos_sin,
                                      void* k_cache, void* v_cache, int layer, int T, int n_q, int n_kv,
                                      int hd, int num_blocks, int block_size, float eps, int kv_fp8,
                                      hipStream_t stream) {
  if (hd > 128 || (hd & 1) || T <= 0) return -2;
  const int n_heads = n_q + 2 * n_kv;
  dim3 grid(T, (n_heads + HEADS_PER_BLOCK - 1) / HEADS_PER_BLOCK);
  if (kv_fp8)
    hipLaunchKernelGGL(qk_norm_rope_kv_kernel<uint8_t>, grid, dim3(256), 0, stream,
                       static_cast<const bf16_t*>(qkv), positions, slots, static_cast<bf16_t*>(q_out),
                       static_cast<const bf16_t*>(q_norm), static_cast<const bf16_t*>(k_norm), cos_sin,
                       static_cast<uint8_t*>(k_cache), static_cast<uint8_t*>(v_cache), layer, T, n_q, n_kv, hd,
                       num_blocks, block_size, eps);
  else
    hipLaunchKernelGGL(qk_norm_rope_kv_kernel<bf16_t>, grid, dim3(256), 0, stream,
                       static_cast<const bf16_t*>(qkv), positions, slots, static_cast<bf16_t*>(q_out),
                       static_cast<const bf16_t*>(q_norm), static_cast<const bf16_t*>(k_norm), cos_sin,
                       static_cast<bf16_t*>(k_cache), static_cast<bf16_t*>(v_cache), layer, T, n_q, n_kv, hd,
                       num_blocks, block_size, eps);
  return BCG_CHECK_LAUNCH();
}
