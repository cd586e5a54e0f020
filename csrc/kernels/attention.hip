// Paged GQA attention on MFMA (v_mfma_f32_16x16x32_bf16) for decode and prefill.
//
// "Swapped" formulation (cdna_hip_programming.md, Appendix B, fused attention):
//   S^T = K · Q^T      A = K rows straight from the paged cache (16 tokens x 32 dims),
//                      B = Q^T fragment held in registers for the whole loop;
//   O^T += V^T · P^T   A = V^T read from the *transposed* V cache ([hd][BS] per
//                      block-head), B = P^T built lane-locally from the S^T
//                      accumulators (no LDS, no shuffles).
// With this orientation every per-query quantity (running max m, sum l, the
// rescale factor, the O^T columns) lives on lane column q = lane & 15, so the
// online softmax needs only two xor-shuffles per chunk and no data movement
// between the two MFMAs.
//
// MFMA 16x16x32 bf16 lane maps (gfx950):
//   A[row = l&15][k = 8(l>>4)+j], B[k = 8(l>>4)+j][col = l&15], C[row = 4(l>>4)+i][col = l&15]
// K-slot permutation used for P/V (same on both operands, so the sum is exact):
//   slot (h, j<4) -> token 4h+j of block 0 of the chunk, (h, j>=4) -> token 4h+j-4 of block 1.
//
// Decode: one workgroup per (sequence, kv head, 256-token split); the G = n_q/n_kv
// query heads of the kv head share every K/V byte (GQA packing: 5 for Qwen3-14B).
// 4 waves x 64 tokens, combined through LDS; splits merged by a second kernel
// (flash-decoding).  Prefill: one workgroup per (64-query tile, query head),
// causal over the cached prefix + the new tokens, varlen via a tile table.

#include "common.h"

namespace {

constexpr int BS = 16;            // KV block size (tokens)
constexpr int SPLIT = 256;        // decode tokens per workgroup
constexpr int DEC_WAVES = 4;
constexpr float LOG2E = 1.4426950408889634f;

struct KVGeom {
  const bf16_t* k;   // [L, NB, n_kv, BS, HD]
  const bf16_t* v;   // [L, NB, n_kv, HD, BS]
  int layer, num_blocks, n_kv;
};

template <int HD>
__device__ __forceinline__ size_t block_base(const KVGeom& g, int blk, int kvh) {
  return ((static_cast<size_t>(g.layer) * g.num_blocks + blk) * g.n_kv + kvh) * (BS * HD);
}

// S^T for one 16-token block: returns C (rows = token 4h+i, col = q).
template <int HD>
__device__ __forceinline__ f32x4 qk_block(const bf16_t* kblock, const bf16x8 (&bq)[HD / 32], int lane) {
  const int r = lane & 15, h = lane >> 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kk = 0; kk < HD / 32; ++kk) {
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(kblock + r * HD + kk * 32 + h * 8);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bq[kk], acc, 0, 0, 0);
  }
  return acc;
}

// One 32-token chunk: online-softmax update + O^T accumulation.
// s0/s1: raw scores of tokens (4h+i) of block 0/1, already scaled to log2 units and masked.
template <int HD>
__device__ __forceinline__ void softmax_pv(f32x4 s0, f32x4 s1, const bf16_t* vb0, const bf16_t* vb1,
                                           bool v0_ok[4], bool v1_ok[4], float& m, float& l,
                                           f32x4 (&o)[HD / 16], int lane) {
  const int r = lane & 15, h = lane >> 4;
  float mx = fmaxf(fmaxf(fmaxf(s0[0], s0[1]), fmaxf(s0[2], s0[3])), fmaxf(fmaxf(s1[0], s1[1]), fmaxf(s1[2], s1[3])));
  mx = fmaxf(mx, __shfl_xor(mx, 16, WAVE));
  mx = fmaxf(mx, __shfl_xor(mx, 32, WAVE));
  // no early exit: the MFMAs below must run with every lane active
  const float m_new = fmaxf(m, mx);
  const bool any = m_new != -INFINITY;
  const float m_use = any ? m_new : 0.f;
  const float alpha = (m == -INFINITY) ? 0.f : exp2f(m - m_use);
  float p[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    p[i] = exp2f(s0[i] - m_use);
    p[4 + i] = exp2f(s1[i] - m_use);
  }
  float ps = ((p[0] + p[1]) + (p[2] + p[3])) + ((p[4] + p[5]) + (p[6] + p[7]));
  ps += __shfl_xor(ps, 16, WAVE);
  ps += __shfl_xor(ps, 32, WAVE);
  l = l * alpha + ps;
  m = m_new;
  bf16x8 bp;
#pragma unroll
  for (int j = 0; j < 8; ++j) bp[j] = static_cast<__bf16>(p[j]);
#pragma unroll
  for (int dt = 0; dt < HD / 16; ++dt) {
    o[dt] *= alpha;
    const int d = dt * 16 + r;
    u16x4 lo = *reinterpret_cast<const u16x4*>(vb0 + d * BS + 4 * h);
    u16x4 hi = *reinterpret_cast<const u16x4*>(vb1 + d * BS + 4 * h);
    u16x8 av;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      av[i] = v0_ok[i] ? lo[i] : static_cast<uint16_t>(0);
      av[4 + i] = v1_ok[i] ? hi[i] : static_cast<uint16_t>(0);
    }
    o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, av), bp, o[dt], 0, 0, 0);
  }
}

// ------------------------------------------------------------------ decode
template <int HD>
__global__ __launch_bounds__(256) void decode_attn_kernel(
    const bf16_t* __restrict__ q, KVGeom g, const int* __restrict__ block_tables, int max_blocks,
    const int* __restrict__ seq_lens, int n_q, float scale_log2, float* __restrict__ part_o,
    float* __restrict__ part_ml, int max_splits) {
  const int split = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int ctx = seq_lens[b];
  const int start = split * SPLIT;
  if (start >= ctx) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, h = lane >> 4;
  const int G = n_q / g.n_kv;
  const int* table = block_tables + static_cast<size_t>(b) * max_blocks;

  // Q^T fragment: col = query head (kvh*G + r), k = dims.
  bf16x8 bq[HD / 32];
  const bool q_ok = r < G;
  const bf16_t* qrow = q + (static_cast<size_t>(b) * n_q + kvh * G + (q_ok ? r : 0)) * HD;
#pragma unroll
  for (int kk = 0; kk < HD / 32; ++kk) {
    u16x8 v = *reinterpret_cast<const u16x8*>(qrow + kk * 32 + h * 8);
    if (!q_ok) v = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    bq[kk] = __builtin_bit_cast(bf16x8, v);
  }

  float m = -INFINITY, l = 0.f;
  f32x4 o[HD / 16];
#pragma unroll
  for (int dt = 0; dt < HD / 16; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int t0 = start + w * 64 + c * 32;
    if (t0 >= ctx) break;
    const int blk0 = table[t0 / BS];
    const int blk1 = (t0 + BS < ctx) ? table[t0 / BS + 1] : blk0;
    const size_t base0 = block_base<HD>(g, blk0, kvh), base1 = block_base<HD>(g, blk1, kvh);
    f32x4 s0 = qk_block<HD>(g.k + base0, bq, lane);
    f32x4 s1 = qk_block<HD>(g.k + base1, bq, lane);
    bool ok0[4], ok1[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ok0[i] = t0 + 4 * h + i < ctx;
      ok1[i] = t0 + BS + 4 * h + i < ctx;
      s0[i] = ok0[i] ? s0[i] * scale_log2 : -INFINITY;
      s1[i] = ok1[i] ? s1[i] * scale_log2 : -INFINITY;
    }
    softmax_pv<HD>(s0, s1, g.v + base0, g.v + base1, ok0, ok1, m, l, o, lane);
  }

  // combine the 4 waves through LDS
  __shared__ float s_ml[DEC_WAVES][2][16];
  __shared__ float s_o[DEC_WAVES][HD][16];
  if (h == 0) {
    s_ml[w][0][r] = m;
    s_ml[w][1][r] = l;
  }
#pragma unroll
  for (int dt = 0; dt < HD / 16; ++dt)
#pragma unroll
    for (int i = 0; i < 4; ++i) s_o[w][dt * 16 + 4 * h + i][r] = o[dt][i];
  __syncthreads();
  for (int idx = threadIdx.x; idx < G * HD; idx += blockDim.x) {
    const int qi = idx / HD, d = idx % HD;
    float mm = -INFINITY;
#pragma unroll
    for (int ww = 0; ww < DEC_WAVES; ++ww) mm = fmaxf(mm, s_ml[ww][0][qi]);
    float ll = 0.f, oo = 0.f;
#pragma unroll
    for (int ww = 0; ww < DEC_WAVES; ++ww) {
      const float mw = s_ml[ww][0][qi];
      const float f = mw == -INFINITY ? 0.f : exp2f(mw - mm);
      ll += s_ml[ww][1][qi] * f;
      oo += s_o[ww][d][qi] * f;
    }
    const size_t pidx = (static_cast<size_t>(b) * n_q + kvh * G + qi) * max_splits + split;
    part_o[pidx * HD + d] = oo;
    if (d == 0) {
      part_ml[pidx * 2] = mm;
      part_ml[pidx * 2 + 1] = ll;
    }
  }
}

template <int HD>
__global__ __launch_bounds__(HD) void decode_combine_kernel(const float* __restrict__ part_o,
                                                            const float* __restrict__ part_ml,
                                                            const int* __restrict__ seq_lens, int n_q,
                                                            int max_splits, bf16_t* __restrict__ out) {
  const int bq = blockIdx.x;  // b * n_q + qh
  const int b = bq / n_q;
  const int d = threadIdx.x;
  const int ns = (seq_lens[b] + SPLIT - 1) / SPLIT;
  const float* ml = part_ml + static_cast<size_t>(bq) * max_splits * 2;
  float mm = -INFINITY;
  for (int s = 0; s < ns; ++s) mm = fmaxf(mm, ml[2 * s]);
  float ll = 0.f, oo = 0.f;
  for (int s = 0; s < ns; ++s) {
    const float f = ml[2 * s] == -INFINITY ? 0.f : exp2f(ml[2 * s] - mm);
    ll += ml[2 * s + 1] * f;
    oo += part_o[(static_cast<size_t>(bq) * max_splits + s) * HD + d] * f;
  }
  out[static_cast<size_t>(bq) * HD + d] = f2bf(ll > 0.f ? oo / ll : 0.f);
}

// ----------------------------------------------------------------- prefill
// tiles[i] = {b, q_begin, q_end} (packed row indices); q rows of sequence b occupy
// [q_start[b], q_start[b+1]) and are its last rows (positions ctx-qlen .. ctx-1).
template <int HD>
__global__ __launch_bounds__(256) void prefill_attn_kernel(
    const bf16_t* __restrict__ q, KVGeom g, const int* __restrict__ block_tables, int max_blocks,
    const int* __restrict__ q_start, const int* __restrict__ seq_lens, const int* __restrict__ tiles,
    int n_q, float scale_log2, bf16_t* __restrict__ out) {
  const int tile = blockIdx.x, qh = blockIdx.y;
  const int b = tiles[3 * tile], q_begin = tiles[3 * tile + 1], q_end = tiles[3 * tile + 2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, h = lane >> 4;
  const int row0 = q_begin + 16 * w;
  if (row0 >= q_end) return;
  const int ctx = seq_lens[b];
  const int qs = q_start[b], qlen = q_start[b + 1] - qs;
  const int pos0 = ctx - qlen;  // position of row qs
  const int kvh = qh / (n_q / g.n_kv);
  const int* table = block_tables + static_cast<size_t>(b) * max_blocks;

  const int my_row = row0 + r;
  const bool row_ok = my_row < q_end;
  const int my_pos = pos0 + (my_row - qs);
  const int last_row = min(row0 + 15, q_end - 1);
  const int kv_end = pos0 + (last_row - qs) + 1;  // exclusive bound of visible keys for this wave

  bf16x8 bq[HD / 32];
  const bf16_t* qrow = q + (static_cast<size_t>(row_ok ? my_row : row0) * n_q + qh) * HD;
#pragma unroll
  for (int kk = 0; kk < HD / 32; ++kk) {
    u16x8 v = *reinterpret_cast<const u16x8*>(qrow + kk * 32 + h * 8);
    if (!row_ok) v = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    bq[kk] = __builtin_bit_cast(bf16x8, v);
  }
  float m = -INFINITY, l = 0.f;
  f32x4 o[HD / 16];
#pragma unroll
  for (int dt = 0; dt < HD / 16; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int t0 = 0; t0 < kv_end; t0 += 32) {
    const int blk0 = table[t0 / BS];
    const int blk1 = (t0 + BS < kv_end) ? table[t0 / BS + 1] : blk0;
    const size_t base0 = block_base<HD>(g, blk0, kvh), base1 = block_base<HD>(g, blk1, kvh);
    f32x4 s0 = qk_block<HD>(g.k + base0, bq, lane);
    f32x4 s1 = qk_block<HD>(g.k + base1, bq, lane);
    bool ok0[4], ok1[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int ta = t0 + 4 * h + i, tb = t0 + BS + 4 * h + i;
      ok0[i] = ta < kv_end;
      ok1[i] = tb < kv_end;
      s0[i] = (ok0[i] && ta <= my_pos) ? s0[i] * scale_log2 : -INFINITY;
      s1[i] = (ok1[i] && tb <= my_pos) ? s1[i] * scale_log2 : -INFINITY;
    }
    softmax_pv<HD>(s0, s1, g.v + base0, g.v + base1, ok0, ok1, m, l, o, lane);
  }
  if (!row_ok) return;
  const float inv = l > 0.f ? 1.f / l : 0.f;
  bf16_t* orow = out + (static_cast<size_t>(my_row) * n_q + qh) * HD;
  // O^T rows d = 16dt + 4h + i are this lane's column (query my_row)
#pragma unroll
  for (int dt = 0; dt < HD / 16; ++dt) {
    u16x4 v;
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = f2bf(o[dt][i] * inv);
    *reinterpret_cast<u16x4*>(orow + dt * 16 + 4 * h) = v;
  }
}

}  // namespace

BCG_API int bcg_decode_workspace_floats(int B, int n_q, int hd, int max_splits) {
  return B * n_q * max_splits * (hd + 2);
}

BCG_API int bcg_paged_attention_decode(const void* q, const void* k_cache, const void* v_cache, int layer,
                                       int num_blocks, int n_kv, const int* block_tables, int max_blocks,
                                       const int* seq_lens, int B, int n_q, int hd, int block_size,
                                       float scale, float* workspace, int max_splits, void* out,
                                       hipStream_t stream) {
  if (block_size != BS || n_q % n_kv || n_q / n_kv > 16 || B <= 0) return -2;
  KVGeom g{static_cast<const bf16_t*>(k_cache), static_cast<const bf16_t*>(v_cache), layer, num_blocks, n_kv};
  float* part_o = workspace;
  float* part_ml = workspace + static_cast<size_t>(B) * n_q * max_splits * hd;
  const float sl = scale * LOG2E;
  dim3 grid(max_splits, n_kv, B);
  if (hd == 128) {
    hipLaunchKernelGGL(decode_attn_kernel<128>, grid, dim3(256), 0, stream, static_cast<const bf16_t*>(q), g,
                       block_tables, max_blocks, seq_lens, n_q, sl, part_o, part_ml, max_splits);
    hipLaunchKernelGGL(decode_combine_kernel<128>, dim3(B * n_q), dim3(128), 0, stream, part_o, part_ml,
                       seq_lens, n_q, max_splits, static_cast<bf16_t*>(out));
  } else if (hd == 64) {
    hipLaunchKernelGGL(decode_attn_kernel<64>, grid, dim3(256), 0, stream, static_cast<const bf16_t*>(q), g,
                       block_tables, max_blocks, seq_lens, n_q, sl, part_o, part_ml, max_splits);
    hipLaunchKernelGGL(decode_combine_kernel<64>, dim3(B * n_q), dim3(64), 0, stream, part_o, part_ml,
                       seq_lens, n_q, max_splits, static_cast<bf16_t*>(out));
  } else {
    return -2;
  }
  return BCG_CHECK_LAUNCH();
}

BCG_API int bcg_paged_attention_prefill(const void* q, const void* k_cache, const void* v_cache, int layer,
                                        int num_blocks, int n_kv, const int* block_tables, int max_blocks,
                                        const int* q_start, const int* seq_lens, const int* tiles, int n_tiles,
                                        int n_q, int hd, int block_size, float scale, void* out,
                                        hipStream_t stream) {
  if (block_size != BS || n_q % n_kv || n_tiles <= 0) return -2;
  KVGeom g{static_cast<const bf16_t*>(k_cache), static_cast<const bf16_t*>(v_cache), layer, num_blocks, n_kv};
  const float sl = scale * LOG2E;
  dim3 grid(n_tiles, n_q);
  if (hd == 128) {
    hipLaunchKernelGGL(prefill_attn_kernel<128>, grid, dim3(256), 0, stream, static_cast<const bf16_t*>(q), g,
                       block_tables, max_blocks, q_start, seq_lens, tiles, n_q, sl, static_cast<bf16_t*>(out));
  } else if (hd == 64) {
    hipLaunchKernelGGL(prefill_attn_kernel<64>, grid, dim3(256), 0, stream, static_cast<const bf16_t*>(q), g,
                       block_tables, max_blocks, q_start, seq_lens, tiles, n_q, sl, static_cast<bf16_t*>(out));
  } else {
    return -2;
  }
  return BCG_CHECK_LAUNCH();
}
