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

#include <type_traits>

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

// Vectorised form (hd = 64 or 128): a lane owns 4 consecutive dims of each half of one head
// (8-B loads and stores instead of 2-B ones), LPH = hd/8 lanes per head, 64/LPH heads per wave,
// the head RMS reduced over the LPH lanes with xor shuffles.  Token metadata (slot,
// position, cos/sin row) is loaded once per lane group.  The one-wave-per-head form above
// moved 2 bytes per lane per access and was latency-bound at decode sizes (34 us per layer
// at 616 rows, ~10x its byte time).
template <typename CacheT, int HD>
__device__ __forceinline__ void rope_kv_token(
    int t, const bf16_t* __restrict__ qkv, const int* __restrict__ positions, const int* __restrict__ slots,
    bf16_t* __restrict__ q_out, const bf16_t* __restrict__ q_norm, const bf16_t* __restrict__ k_norm,
    const float* __restrict__ cos_sin, CacheT* __restrict__ k_cache, CacheT* __restrict__ v_cache,
    int layer, int n_q, int n_kv, int num_blocks, int block_size, float eps, int skip_v) {
  constexpr int HALF = HD / 2, LPH = HALF / 4, HPW = 64 / LPH;  // lanes per head, heads per wave
  const int lane = threadIdx.x & 63, li = lane % LPH;
  const int slot_head = (blockIdx.y * 4 + (threadIdx.x >> 6)) * HPW + lane / LPH;
  const int n_heads = n_q + 2 * n_kv;
  const bool valid = slot_head < n_heads;  // idle lanes still take part in the shuffles
  const int d0 = 4 * li;
  const bf16_t* src = qkv + (static_cast<size_t>(t) * n_heads + (valid ? slot_head : 0)) * HD;
  u16x4 a = *reinterpret_cast<const u16x4*>(src + d0), bv = *reinterpret_cast<const u16x4*>(src + HALF + d0);
  float x1[4], x2[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) x1[e] = bf2f(a[e]), x2[e] = bf2f(bv[e]);
  const int slot = slots[t];
  const int blk = slot / block_size, off = slot % block_size;

  if (slot_head >= n_q + n_kv) {  // value head (or idle): transposed store, no transform
    if (!valid || skip_v) return;  // skip_v: v_write_group_kernel stores V
    const int h = slot_head - n_q - n_kv;
    CacheT* vb = v_cache + ((static_cast<size_t>(layer) * num_blocks + blk) * n_kv + h) * HD * block_size + off;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      vb[static_cast<size_t>(d0 + e) * block_size] = to_cache<CacheT>(x1[e]);
      vb[static_cast<size_t>(HALF + d0 + e) * block_size] = to_cache<CacheT>(x2[e]);
    }
    return;
  }
  // (the branch above is uniform per lane group; the shuffles below stay within a group
  //  of query/key heads, whose lanes all reach them)
  const bool is_q = slot_head < n_q;
  const bf16_t* nw = is_q ? q_norm : k_norm;
  if (nw != nullptr) {
    float ss = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) ss += x1[e] * x1[e] + x2[e] * x2[e];
#pragma unroll
    for (int o = LPH / 2; o >= 1; o >>= 1) ss += __shfl_xor(ss, o, 64);
    const float inv = rsqrtf(ss / HD + eps);
    const u16x4 w1 = *reinterpret_cast<const u16x4*>(nw + d0), w2 = *reinterpret_cast<const u16x4*>(nw + HALF + d0);
#pragma unroll
    for (int e = 0; e < 4; ++e) x1[e] *= inv * bf2f(w1[e]), x2[e] *= inv * bf2f(w2[e]);
  }
  const float* cs = cos_sin + static_cast<size_t>(positions[t]) * HD;
  const f32x4 c = *reinterpret_cast<const f32x4*>(cs + d0), sn = *reinterpret_cast<const f32x4*>(cs + HALF + d0);
  float y1[4], y2[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) y1[e] = x1[e] * c[e] - x2[e] * sn[e], y2[e] = x2[e] * c[e] + x1[e] * sn[e];
  if (is_q) {
    bf16_t* dst = q_out + (static_cast<size_t>(t) * n_q + slot_head) * HD;
    u16x4 o1, o2;
#pragma unroll
    for (int e = 0; e < 4; ++e) o1[e] = f2bf(y1[e]), o2[e] = f2bf(y2[e]);
    *reinterpret_cast<u16x4*>(dst + d0) = o1;
    *reinterpret_cast<u16x4*>(dst + HALF + d0) = o2;
  } else {
    const int h = slot_head - n_q;
    CacheT* dst = k_cache + (((static_cast<size_t>(layer) * num_blocks + blk) * n_kv + h) * block_size + off) * HD;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      dst[d0 + e] = to_cache<CacheT>(y1[e]);
      dst[HALF + d0 + e] = to_cache<CacheT>(y2[e]);
    }
  }
}

// ROPE_TPB consecutive tokens per workgroup: a prefill chunk launched one token per workgroup
// was ~49k workgroups of 8 KB each (Qwen3-14B, 16k tokens) -- dispatch-bound, not byte-bound.
constexpr int ROPE_TPB = 4;

template <typename CacheT, int HD>
__global__ __launch_bounds__(256) void qk_norm_rope_kv_vec_kernel(
    const bf16_t* __restrict__ qkv, const int* __restrict__ positions, const int* __restrict__ slots,
    bf16_t* __restrict__ q_out, const bf16_t* __restrict__ q_norm, const bf16_t* __restrict__ k_norm,
    const float* __restrict__ cos_sin, CacheT* __restrict__ k_cache, CacheT* __restrict__ v_cache,
    int layer, int T, int n_q, int n_kv, int num_blocks, int block_size, float eps, int skip_v, int tpb) {
  const int t0 = blockIdx.x * tpb, t1 = min(T, t0 + tpb);
  for (int t = t0; t < t1; ++t)  // block-uniform
    rope_kv_token<CacheT, HD>(t, qkv, positions, slots, q_out, q_norm, k_norm, cos_sin, k_cache, v_cache, layer,
                              n_q, n_kv, num_blocks, block_size, eps, skip_v);
}

// Prefill V (T >= 64): one workgroup per (16 consecutive tokens, kv head), one thread per dim.
// When the 16 tokens fill one KV block in order (the common case inside a prompt), thread d
// gathers its 16 values and writes the block's V^T row d as 32 contiguous bytes -- the
// per-token form writes 2 bytes at a 32-B stride per element (418 -> 286 us per layer at
// 16k tokens was left mostly in those stores).  Other groups store element by element.
//
// The block is 2*HD threads and both sides move 16 B per lane: thread (i = tid / (HD/8),
// c = tid % (HD/8)) loads dims 8c..8c+7 of token i (one 16-B load; the former one-thread-per-dim
// form issued 16 two-byte loads per thread, 128 B per wave instruction, and ran at ~1.4 TB/s),
// the 16 x HD tile is transposed through LDS, and thread (d = tid / 2, half) stores tokens
// 8*half..8*half+7 of V^T row d as one 16-B store.
template <int HD>
__global__ __launch_bounds__(2 * HD) void v_write_group_kernel(const bf16_t* __restrict__ qkv,
                                                               const int* __restrict__ slots,
                                                               bf16_t* __restrict__ v_cache, int layer, int T,
                                                               int n_q, int n_kv, int num_blocks, int block_size) {
  constexpr int CPT = HD / 8;      // 16-B chunks per token row
  constexpr int LD = HD + 8;       // LDS row pitch (bf16): rows start 16 B apart in the bank map
  __shared__ __attribute__((aligned(16))) uint16_t tile[16][LD];
  const int t0 = blockIdx.x * 16, h = blockIdx.y, tid = threadIdx.x;
  const int nt = min(16, T - t0);
  const int n_heads = n_q + 2 * n_kv;
  const int s0 = slots[t0];
  const bool mine = tid >= nt || slots[t0 + tid] == s0 + tid;  // thread i < 16 checks token i
  const bool fast = __syncthreads_and(mine) && nt == 16 && block_size == 16 && s0 % 16 == 0;
  const bf16_t* head = qkv + static_cast<size_t>(t0) * n_heads * HD + static_cast<size_t>(n_q + n_kv + h) * HD;
  if (fast) {
    const int i = tid / CPT, c = tid % CPT;
    const u16x8 x = *reinterpret_cast<const u16x8*>(head + static_cast<size_t>(i) * n_heads * HD + 8 * c);
    *reinterpret_cast<u16x8*>(&tile[i][8 * c]) = x;
    __syncthreads();
    const int d = tid >> 1, half = tid & 1;
    uint32_t w[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      w[j] = uint32_t(tile[8 * half + 2 * j][d]) | (uint32_t(tile[8 * half + 2 * j + 1][d]) << 16);
    const int blk = s0 / 16;
    uint4* dst = reinterpret_cast<uint4*>(v_cache + ((static_cast<size_t>(layer) * num_blocks + blk) * n_kv + h) * HD * 16 +
                                          static_cast<size_t>(d) * 16 + 8 * half);
    *dst = uint4{w[0], w[1], w[2], w[3]};
    return;
  }
  if (tid >= HD) return;  // element-wise path: one thread per dim
  const int d = tid;
  const bf16_t* src = head + d;
  for (int i = 0; i < nt; ++i) {
    const int slot = slots[t0 + i];
    const int blk = slot / block_size, off = slot % block_size;
    v_cache[((static_cast<size_t>(layer) * num_blocks + blk) * n_kv + h) * HD * block_size +
            static_cast<size_t>(d) * block_size + off] = src[static_cast<size_t>(i) * n_heads * HD];
  }
}

template <typename CacheT, int HD>
void launch_vec(const void* qkv, const int* positions, const int* slots, void* q_out, const void* q_norm,
                const void* k_norm, const float* cos_sin, void* k_cache, void* v_cache, int layer, int T, int n_q,
                int n_kv, int num_blocks, int block_size, float eps, int contiguous, hipStream_t stream) {
  constexpr int HPB = 4 * (64 / (HD / 8));  // heads per 256-thread block
  const int n_heads = n_q + 2 * n_kv;
  // contiguous = 0 (decode: one token per sequence): no group ever fills a block, and the grouped
  // writer's element-wise path walked its 16 tokens one after another (13.6 us per layer at 768
  // rows against ~1 us of transposed stores inside the rope kernel)
  const bool group_v = std::is_same<CacheT, bf16_t>::value && T >= 64 && contiguous;
  // group_v: v_write_group_kernel stores V, so the grid covers the query/key heads only (a
  // block past them would load its V rows just to return: Qwen3-14B's fourth head block, 2 KB
  // per token); V heads inside the last query/key block still return early through skip_v
  const int grid_heads = group_v ? n_q + n_kv : n_heads;
  const int tpb = T >= 1024 ? ROPE_TPB : 1;  // decode rows keep one token per workgroup (parallelism)
  hipLaunchKernelGGL((qk_norm_rope_kv_vec_kernel<CacheT, HD>), dim3((T + tpb - 1) / tpb, (grid_heads + HPB - 1) / HPB),
                     dim3(256), 0,
                     stream, static_cast<const bf16_t*>(qkv), positions, slots, static_cast<bf16_t*>(q_out),
                     static_cast<const bf16_t*>(q_norm), static_cast<const bf16_t*>(k_norm), cos_sin,
                     static_cast<CacheT*>(k_cache), static_cast<CacheT*>(v_cache), layer, T, n_q, n_kv, num_blocks,
                     block_size, eps, group_v ? 1 : 0, tpb);
  if (group_v)
    hipLaunchKernelGGL((v_write_group_kernel<HD>), dim3((T + 15) / 16, n_kv), dim3(2 * HD), 0, stream,
                       static_cast<const bf16_t*>(qkv), slots, reinterpret_cast<bf16_t*>(v_cache), layer, T, n_q,
                       n_kv, num_blocks, block_size);
}

}  // namespace

BCG_API int bcg_qk_norm_rope_kv_write(const void* qkv, const int* positions, const int* slots, void* q_out,
                                      const void* q_norm, const void* k_norm, const float* cos_sin,
                                      void* k_cache, void* v_cache, int layer, int T, int n_q, int n_kv,
                                      int hd, int num_blocks, int block_size, float eps, int kv_fp8,
                                      int contiguous, hipStream_t stream) {
  if (hd > 128 || (hd & 1) || T <= 0) return -2;
  if (hd == 128 || hd == 64) {
    if (kv_fp8) {
      if (hd == 128)
        launch_vec<uint8_t, 128>(qkv, positions, slots, q_out, q_norm, k_norm, cos_sin, k_cache, v_cache, layer, T,
                                 n_q, n_kv, num_blocks, block_size, eps, contiguous, stream);
      else
        launch_vec<uint8_t, 64>(qkv, positions, slots, q_out, q_norm, k_norm, cos_sin, k_cache, v_cache, layer, T,
                                n_q, n_kv, num_blocks, block_size, eps, contiguous, stream);
    } else {
      if (hd == 128)
        launch_vec<bf16_t, 128>(qkv, positions, slots, q_out, q_norm, k_norm, cos_sin, k_cache, v_cache, layer, T,
                                n_q, n_kv, num_blocks, block_size, eps, contiguous, stream);
      else
        launch_vec<bf16_t, 64>(qkv, positions, slots, q_out, q_norm, k_norm, cos_sin, k_cache, v_cache, layer, T,
                               n_q, n_kv, num_blocks, block_size, eps, contiguous, stream);
    }
    return BCG_CHECK_LAUNCH();
  }
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
