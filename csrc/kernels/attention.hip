// Paged GQA attention on MFMA (v_mfma_f32_16x16x32_bf16) for decode and prefill.
//
// "Swapped" formulation (cdna_hip_programming.md, Appendix B, fused attention):
//   S^T = K · Q^T      A = K rows straight from the paged cache (16 tokens x 32 dims),
//                      B = Q^T fragment held in registers for the whole loop;
//   O^T += V^T · P^T   A = V^T read from the *transposed* V cache ([hd][BS] per
//                      block-head), B = P^T built lane-locally from the S^T
//                      accumulators (no LDS, no shuffles).
// Every per-query quantity (running max m, sum l, rescale factor, O^T column)
// lives on lane column q = lane & 15: the online softmax needs two
// xor-shuffles per 32-token chunk and no data movement between the MFMAs.
//
// MFMA 16x16x32 bf16 lane maps (gfx950):
//   A[row = l&15][k = 8(l>>4)+j], B[k = 8(l>>4)+j][col = l&15], C[row = 4(l>>4)+i][col = l&15]
// Token permutation of a 32-token chunk (makes every V fragment ONE 16-byte load):
//   S^T tile u (u = 0,1), C row 4h+i  <->  chunk token 8h + 4u + i
//   so lane group h holds the scores of tokens 8h..8h+7, which is exactly the
//   k-slot order (h, j) <-> token 8h+j of the P^T / V^T operands; tokens 8h..8h+7
//   are 16 contiguous bytes of one V^T row (block h>>1, offset 8(h&1)).
//   K tiles load row r from token 8(r>>2) + 4u + (r&3) (a row gather: free).
//
// Decode: one workgroup per (sequence, kv head, 256-token split); the G = n_q/n_kv query
// heads of the kv head share every K/V byte (GQA packing: 5 for Qwen3-14B);
// waves are combined through LDS and splits merged by a second kernel
// (flash-decoding).  Prefill: one workgroup per (64-query tile, query
// head), causal over cached prefix + new tokens, varlen via a tile table.

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "common.h"

namespace {

constexpr int BS = 16;            // KV block size (tokens)
constexpr int DEC_WAVES = 4;
constexpr int CHUNK = 32;
constexpr float LOG2E = 1.4426950408889634f;
constexpr float RESCALE_LOG2 = 8.f;  // lazy online-softmax rescale threshold (log2 units)

// 2^x as the bare v_exp_f32.  exp2f() wraps it in a denormal range reduction (v_cmp +
// v_cndmask + v_ldexp around every exponential: ~3 extra VALU per score); softmax
// arguments are <= 0 here and a result below 2^-126 may flush to 0.
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Single-instruction maxima.  fmaxf() on MFMA results makes hipcc canonicalise every input
// first (one v_max_f32 x, x per score: 32 extra VALU per 64 MFMAs in the prefill loop); the
// scores here are never NaN, so the raw v_max3 / v_max forms are exact.
__device__ __forceinline__ float vmax3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}
__device__ __forceinline__ float vmax(float a, float b) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
typedef float f32x2 __attribute__((ext_vector_type(2)));

struct KVGeom {
  const bf16_t* k;   // [L, NB, n_kv, BS, HD]
  const bf16_t* v;   // [L, NB, n_kv, HD, BS]
  int layer, num_blocks, n_kv;
};

template <int HD>
__device__ __forceinline__ size_t block_base(const KVGeom& g, int blk, int kvh) {
  return ((static_cast<size_t>(g.layer) * g.num_blocks + blk) * g.n_kv + kvh) * (BS * HD);
}

// A chunk's operands as loaded: bf16x8 (16 B) per fragment, or -- fp8 KV cache --
// the raw 8 e4m3fn bytes, widened to bf16 only right before their MFMA so the
// loads of the next chunk stay in flight (converting at load time would wait).
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int HD, bool F8 = false>
struct Chunk {
  typedef typename std::conditional<F8, u32x2, bf16x8>::type E;
  E k[2][HD / 32];   // S^T A-operands, tile u, k-step kk
  E v[HD / 16];      // O^T A-operands, d-tile dt
};

__device__ __forceinline__ bf16x8 to_bf16x8(const bf16x8& x) { return x; }

__device__ __forceinline__ bf16x8 to_bf16x8(const u32x2& x) {  // 8 x e4m3fn -> 8 x bf16 (exact)
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  const bf16x2 a = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(x[0], 1.f, false);
  const bf16x2 b = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(x[0], 1.f, true);
  const bf16x2 c = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(x[1], 1.f, false);
  const bf16x2 d = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(x[1], 1.f, true);
  return bf16x8{a[0], a[1], b[0], b[1], c[0], c[1], d[0], d[1]};
}

// Issue every load of one 32-token chunk whose blocks are blk0/blk1.
template <int HD, bool F8 = false>
__device__ __forceinline__ void load_chunk(Chunk<HD, F8>& c, const KVGeom& g, int blk0, int blk1, int kvh,
                                           int lane) {
  typedef typename Chunk<HD, F8>::E E;
  typedef typename std::conditional<F8, uint8_t, bf16_t>::type T;  // cache element
  const T* kc = reinterpret_cast<const T*>(g.k);
  const T* vc = reinterpret_cast<const T*>(g.v);
  const int r = lane & 15, h = lane >> 4;
  const size_t b0 = block_base<HD>(g, blk0, kvh), b1 = block_base<HD>(g, blk1, kvh);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int t = 8 * (r >> 2) + 4 * u + (r & 3);
    const T* krow = kc + (t < BS ? b0 : b1) + (t & (BS - 1)) * HD + 8 * h;
#pragma unroll
    for (int kk = 0; kk < HD / 32; ++kk) c.k[u][kk] = *reinterpret_cast<const E*>(krow + kk * 32);
  }
  const T* vb = vc + (h < 2 ? b0 : b1) + 8 * (h & 1);
#pragma unroll
  for (int dt = 0; dt < HD / 16; ++dt) c.v[dt] = *reinterpret_cast<const E*>(vb + (dt * 16 + r) * BS);
  // Keep all 16 loads of the chunk together: without this fence hipcc sinks the
  // V loads below the S^T MFMAs that wait for K, i.e. two serial HBM round trips.
  __builtin_amdgcn_sched_barrier(0);
}

// The K half / V half of load_chunk, for loops that reload a chunk's registers in place
// (K right after the S^T MFMAs consumed it, V after the P.V MFMAs).
template <int HD, bool F8 = false>
__device__ __forceinline__ void load_chunk_k(Chunk<HD, F8>& c, const KVGeom& g, int blk0, int blk1, int kvh,
                                             int lane) {
  typedef typename Chunk<HD, F8>::E E;
  typedef typename std::conditional<F8, uint8_t, bf16_t>::type T;
  const T* kc = reinterpret_cast<const T*>(g.k);
  const int r = lane & 15, h = lane >> 4;
  const size_t b0 = block_base<HD>(g, blk0, kvh), b1 = block_base<HD>(g, blk1, kvh);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int t = 8 * (r >> 2) + 4 * u + (r & 3);
    const T* krow = kc + (t < BS ? b0 : b1) + (t & (BS - 1)) * HD + 8 * h;
#pragma unroll
    for (int kk = 0; kk < HD / 32; ++kk) c.k[u][kk] = *reinterpret_cast<const E*>(krow + kk * 32);
  }
}

template <int HD, bool F8 = false>
__device__ __forceinline__ void load_chunk_v(Chunk<HD, F8>& c, const KVGeom& g, int blk0, int blk1, int kvh,
                                             int lane) {
  typedef typename Chunk<HD, F8>::E E;
  typedef typename std::conditional<F8, uint8_t, bf16_t>::type T;
  const T* vc = reinterpret_cast<const T*>(g.v);
  const int r = lane & 15, h = lane >> 4;
  const T* vb = vc + block_base<HD>(g, h < 2 ? blk0 : blk1, kvh) + 8 * (h & 1);
#pragma unroll
  for (int dt = 0; dt < HD / 16; ++dt) c.v[dt] = *reinterpret_cast<const E*>(vb + (dt * 16 + r) * BS);
}

// Reductions over the 4 lane rows (h = lane >> 4) that share a query column:
// v_permlane16_swap (rows 0<->1, 2<->3) then v_permlane32_swap (0<->2, 1<->3),
// two VALU ops each instead of ds_bpermute round trips through the LDS
// crossbar (~100 cycles apiece, four of them in series per chunk).  Both
// halves of each swap are combined, so every lane gets identical bits.
__device__ __forceinline__ float rows_max(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = vmax(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return vmax(__uint_as_float(b[0]), __uint_as_float(b[1]));
}

__device__ __forceinline__ float rows_sum(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// Online-softmax update + O^T accumulation for one chunk starting at token t0.
// visible(t) decides masking (t = absolute token index); kv_end bounds V reads.
// MASKED = false: the caller guarantees every token of the chunk is visible to
// every column (wave-uniform), so the per-token mask and the V-tail zeroing
// (~60 VALU ops per chunk beside 16 MFMAs) are skipped.
template <int HD, typename Vis, bool MASKED = true, bool F8 = false, bool LAZY = true>
__device__ __forceinline__ void compute_chunk(const Chunk<HD, F8>& c, const bf16x8 (&bq)[HD / 32], int t0, int kv_end,
                                              Vis visible, float scale_log2, float& m, float& l,
                                              f32x4 (&o)[HD / 16], int lane) {
  const int h = lane >> 4;
  f32x4 s[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    s[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < HD / 32; ++kk)
      s[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(to_bf16x8(c.k[u][kk]), bq[kk], s[u], 0, 0, 0);
  }
  float p[8];
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int t = t0 + 8 * h + j;
    const float sv = s[j >> 2][j & 3];
    p[j] = (!MASKED || (t < kv_end && visible(t))) ? sv * scale_log2 : -INFINITY;
    mx = fmaxf(mx, p[j]);
  }
  mx = rows_max(mx);
  // Lazy rescale: the reference max m only moves when some column's chunk max
  // exceeds it by more than 2^RESCALE_LOG2 (then P <= 2^8 stays exact in fp32 /
  // bf16 and l cannot overflow over an 8k context).  Rescaling O is 32 VALU
  // multiplies plus the accumulator moves around them -- the kernels were
  // VALU-bound on it (14 VALU per MFMA, PMC); after the first chunks it is rare.
  if constexpr (LAZY) {
    if (__builtin_amdgcn_ballot_w64(mx > m + RESCALE_LOG2) != 0) {  // wave-uniform
      const float m_new = fmaxf(m, mx);
      const float alpha = m == -INFINITY ? 0.f : fast_exp2(m - m_new);
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < HD / 16; ++dt) o[dt] *= alpha;
      m = m_new;
    }
  }
  // eager (LAZY = false): rescale every chunk, O folded into the P.V loop below --
  // the branch-free form keeps fewer registers live (no spills at NT = 4)
  float alpha = 1.f;
  if constexpr (!LAZY) {
    const float m_new = fmaxf(m, mx);
    alpha = m == -INFINITY ? 0.f : fast_exp2(m - (m_new == -INFINITY ? 0.f : m_new));
    l *= alpha;
    m = m_new;
  }
  const float m_use = m == -INFINITY ? 0.f : m;
  float ps = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    p[j] = fast_exp2(p[j] - m_use);
    ps += p[j];
  }
  ps = rows_sum(ps);
  l += ps;
  bf16x8 bp;
#pragma unroll
  for (int j = 0; j < 8; ++j) bp[j] = static_cast<__bf16>(p[j]);
  // tokens past kv_end may hold stale (even non-finite) bytes: zero their V
  // with branch-free 32-bit masks (a divergent branch here splits the vmcnt waits)
  if constexpr (MASKED) {
    uint32_t keep[4];
#pragma unroll
    for (int j2 = 0; j2 < 4; ++j2) {
      const int t = t0 + 8 * h + 2 * j2;
      keep[j2] = (t < kv_end ? 0x0000ffffu : 0u) | (t + 1 < kv_end ? 0xffff0000u : 0u);
    }
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) {
      if constexpr (!LAZY) o[dt] *= alpha;
      u32x4 va = __builtin_bit_cast(u32x4, to_bf16x8(c.v[dt]));
#pragma unroll
      for (int j2 = 0; j2 < 4; ++j2) va[j2] &= keep[j2];
      o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, va), bp, o[dt], 0, 0, 0);
    }
  } else {
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) {
      if constexpr (!LAZY) o[dt] *= alpha;
      o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(to_bf16x8(c.v[dt]), bp, o[dt], 0, 0, 0);
    }
  }
}


// All NT query sub-tiles of a wave on one chunk that every row of every sub-tile sees in
// full (no mask), as ONE straight-line block: the S^T MFMAs of every sub-tile first, then
// each sub-tile's softmax (its VALU runs while the later sub-tiles' MFMAs are still in the
// pipe), then every P.V MFMA.  Split in two so the caller's loop can leave for the (rare,
// lazy: only when some column's running max moves by > 2^RESCALE_LOG2) rescale of O:
//   full_scores  S^T MFMAs, the next chunk's K reloaded in place, per-column chunk max;
//                returns whether any column needs a rescale (wave-uniform);
//   full_pv      P = exp2(S - m), l += rowsum(P), O^T += V^T P^T, next chunk's V reloaded.
// With the rescale (VALU on the O accumulators) inside the loop body, hipcc copied all
// 128 O accumulators AGPR -> VGPR at the top of EVERY chunk, taken or not (128
// v_accvgpr_read per 64 MFMAs at NT = 4); outside it, O stays in AGPRs.
template <int HD, int NT, bool F8, typename ReloadK>
__device__ __forceinline__ bool full_scores(Chunk<HD, F8>& c, const bf16x8 (&bq)[NT][HD / 32], float scale_log2,
                                            const float (&m)[NT], f32x2 (&t)[NT][4], float (&mx)[NT],
                                            ReloadK reload_k) {
  f32x4 s[NT][2];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      s[nt][u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < HD / 32; ++kk)
        s[nt][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(to_bf16x8(c.k[u][kk]), bq[nt][kk], s[nt][u], 0, 0, 0);
    }
  reload_k(c);  // next chunk's K into the registers the S^T MFMAs just read
  // every score is read from the MFMA result ONCE: t = S * scale - m (two per v_pk_fma_f32), its
  // column max decides the lazy rescale, and full_pv exponentiates t directly
  // (before the first chunk m = -inf: t is taken relative to 0 and the chunk always rescales)
  bool grow = false;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const bool first = m[nt] == -INFINITY;
    const float m_eff = first ? 0.f : m[nt];
    const f32x2 sc = {scale_log2, scale_log2}, mm = {m_eff, m_eff};
#pragma unroll
    for (int q = 0; q < 4; ++q)
      t[nt][q] = f32x2{s[nt][q >> 1][2 * (q & 1)], s[nt][q >> 1][2 * (q & 1) + 1]} * sc - mm;
    const float v = vmax3(vmax3(t[nt][0].x, t[nt][0].y, t[nt][1].x), vmax3(t[nt][1].y, t[nt][2].x, t[nt][2].y),
                          vmax(t[nt][3].x, t[nt][3].y));
    const float rel = rows_max(v);  // chunk max relative to the running max
    mx[nt] = rel + m_eff;
    grow |= first || rel > RESCALE_LOG2;
  }
  return __builtin_amdgcn_ballot_w64(grow) != 0;
}

template <int HD, int NT, bool F8, typename ReloadV>
__device__ __forceinline__ void full_pv(Chunk<HD, F8>& c, const f32x2 (&t)[NT][4], float (&l)[NT],
                                        f32x4 (&o)[NT][HD / 16], ReloadV reload_v) {
  bf16x8 bp[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    f32x2 p[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      p[q] = f32x2{fast_exp2(t[nt][q].x), fast_exp2(t[nt][q].y)};
      bp[nt][2 * q] = static_cast<__bf16>(p[q].x);
      bp[nt][2 * q + 1] = static_cast<__bf16>(p[q].y);
    }
    const f32x2 ps2 = (p[0] + p[1]) + (p[2] + p[3]);  // packed adds
    l[nt] += rows_sum(ps2.x + ps2.y);
  }
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt)
      o[nt][dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(to_bf16x8(c.v[dt]), bp[nt], o[nt][dt], 0, 0, 0);
  reload_v(c);
}

// The (rare) lazy rescale: the running max moves to the chunk max; O and l scale by 2^(m - m_new)
// and the chunk's relative scores t shift by the same amount.
template <int HD, int NT>
__device__ __forceinline__ void full_rescale(const float (&mx)[NT], float (&m)[NT], float (&l)[NT],
                                             f32x4 (&o)[NT][HD / 16], f32x2 (&t)[NT][4]) {
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const bool first = m[nt] == -INFINITY;
    const float m_new = first ? mx[nt] : fmaxf(m[nt], mx[nt]);
    const float alpha = first ? 0.f : fast_exp2(m[nt] - m_new);
    l[nt] *= alpha;
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) o[nt][dt] *= alpha;
    const float shift = m_new - (first ? 0.f : m[nt]);  // t was relative to m_eff (full_scores)
    const f32x2 sh = {shift, shift};
#pragma unroll
    for (int q = 0; q < 4; ++q) t[nt][q] -= sh;
    m[nt] = m_new;
  }
}

template <int HD>
__device__ __forceinline__ void load_q(bf16x8 (&bq)[HD / 32], const bf16_t* row, bool ok, int lane) {
  const int h = lane >> 4;
#pragma unroll
  for (int kk = 0; kk < HD / 32; ++kk) {
    u16x8 v = *reinterpret_cast<const u16x8*>(row + kk * 32 + h * 8);
    if (!ok) v = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    bq[kk] = __builtin_bit_cast(bf16x8, v);
  }
}

struct AllVisible {
  __device__ bool operator()(int) const { return true; }
};

struct Causal {
  int pos;
  __device__ bool operator()(int t) const { return t <= pos; }
};

// ------------------------------------------------------------------ decode
// Work item = (sequence b, CPW*128-token split, kv head): the 4 waves of a
// workgroup take CPW consecutive 32-token chunks each (all CPW x 16 16-B loads
// issued before the first MFMA), and the G = n_q / n_kv query heads of the kv head
// share every K/V byte (GQA packing).  Items are enumerated from the LIVE
// context lengths -- a prefix sum over ceil(ctx_b / split) computed by every
// workgroup into LDS -- and a fixed grid strides over them.  A grid sized from
// the block-table width instead (graph-safe, but ctx << max_model_len) spent
// most of its workgroups reading seq_lens only to exit: 78 % of the launch at
// B = 160, ctx 1700, max_model_len 8192.
constexpr int DEC_MAX_B = 2048;

//
// Shared-prefix (cascade) form: rows whose leading blocks are the SAME physical blocks
// (prefix cache: an agent's system prompt, identical in every game) get kv_begin[b] =
// the shared token count and split_base[b] = the shared pass's split count.
// decode_shared_kernel computes their attention over the shared blocks once per group --
// every member's query heads packed into MFMA columns, each shared K/V byte read once per
// 64 columns instead of once per row -- into slots 0 .. split_base-1; this kernel covers
// [kv_begin, ctx) into the slots after them; the combine merges all slots.
// kv_begin == nullptr: no cascade (every row from token 0).
template <int HD, bool F8 = false, int CPW = 1>
__global__ __launch_bounds__(256) void decode_attn_kernel(
    const bf16_t* __restrict__ q, KVGeom g, const int* __restrict__ block_tables, int max_blocks,
    const int* __restrict__ seq_lens, int B, int n_q, float scale_log2, float* __restrict__ part_o,
    float* __restrict__ part_ml, int max_splits, const int* __restrict__ kv_begin,
    const int* __restrict__ split_base) {
  // CPW chunks per wave: an item covers DEC_WAVES * CPW * 32 tokens; every chunk's loads of
  // a wave are issued before its first MFMA (CPW x 16 loads in flight per wave), and the
  // split partials / merge traffic shrink by CPW
  constexpr int DEC_SPLIT = DEC_WAVES * CHUNK * CPW;
  __shared__ int s_pre[DEC_MAX_B + 1];
  __shared__ int s_wsum[DEC_WAVES];
  __shared__ float s_ml[DEC_WAVES][2][16];
  __shared__ float s_o[DEC_WAVES][HD][16 + 1];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 15, h = lane >> 4;
  const int G = n_q / g.n_kv;

  // ---- item enumeration: s_pre[b] = sum_{b' < b} ceil(ctx_b' / 128)
  {
    constexpr int PER_MAX = DEC_MAX_B / 256;
    const int per = (B + 255) / 256;  // <= PER_MAX
    int cnt[PER_MAX], sum = 0;
#pragma unroll
    for (int j = 0; j < PER_MAX; ++j) {
      const int i = tid * per + j;
      const int own = (j < per && i < B) ? max(0, seq_lens[i] - (kv_begin ? kv_begin[i] : 0)) : 0;
      cnt[j] = (own + DEC_SPLIT - 1) / DEC_SPLIT;
      sum += cnt[j];
    }
    int incl = sum;  // inclusive wave scan
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int v = __shfl_up(incl, o, WAVE);
      if (lane >= o) incl += v;
    }
    if (lane == 63) s_wsum[w] = incl;
    __syncthreads();
    int base = incl - sum;
    for (int ww = 0; ww < w; ++ww) base += s_wsum[ww];
#pragma unroll
    for (int j = 0; j < PER_MAX; ++j) {
      const int i = tid * per + j;
      if (j < per && i < B) s_pre[i] = base;
      base += cnt[j];
    }
    if (tid == 255) s_pre[B] = base;
    __syncthreads();
  }
  const int n_items = s_pre[B] * g.n_kv;

  for (int item = blockIdx.x; item < n_items; item += gridDim.x) {
    const int pos = item / g.n_kv, kvh = item - pos * g.n_kv;
    int lo = 0, hi = B - 1;  // last b with s_pre[b] <= pos (binary search, wave-uniform)
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (s_pre[mid] <= pos) lo = mid; else hi = mid - 1;
    }
    const int b = lo, split = pos - s_pre[b];
    const int ctx = seq_lens[b];
    const int start = (kv_begin ? kv_begin[b] : 0) + split * DEC_SPLIT;
    const int slot = (split_base ? split_base[b] : 0) + split;  // after the shared-pass slots
    const int* table = block_tables + static_cast<size_t>(b) * max_blocks;

    bf16x8 bq[HD / 32];
    load_q<HD>(bq, q + (static_cast<size_t>(b) * n_q + kvh * G + (r < G ? r : 0)) * HD, r < G, lane);
    float m = -INFINITY, l = 0.f;
    f32x4 o[HD / 16];
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) o[dt] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int t0 = start + w * CHUNK * CPW;
    const int last_blk = (ctx - 1) / BS;
    Chunk<HD, F8> c[CPW];
#pragma unroll
    for (int j = 0; j < CPW; ++j) {
      const int tj = t0 + j * CHUNK;
      if (tj < ctx)  // wave-uniform
        load_chunk<HD, F8>(c[j], g, table[tj / BS], table[min(tj / BS + 1, last_blk)], kvh, lane);
    }
#pragma unroll
    for (int j = 0; j < CPW; ++j) {
      const int tj = t0 + j * CHUNK;
      if (tj >= ctx) break;  // wave-uniform
      if (tj + CHUNK <= ctx)  // wave-uniform: a full chunk needs no tail masking
        compute_chunk<HD, AllVisible, false, F8>(c[j], bq, tj, ctx, AllVisible{}, scale_log2, m, l, o, lane);
      else
        compute_chunk<HD, AllVisible, true, F8>(c[j], bq, tj, ctx, AllVisible{}, scale_log2, m, l, o, lane);
    }

    // combine the 4 waves through LDS
    if (h == 0) {
      s_ml[w][0][r] = m;
      s_ml[w][1][r] = l;
    }
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt)
#pragma unroll
      for (int i = 0; i < 4; ++i) s_o[w][dt * 16 + 4 * h + i][r] = o[dt][i];
    __syncthreads();
    for (int idx = tid; idx < G * HD; idx += blockDim.x) {
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
      const size_t pidx = (static_cast<size_t>(b) * n_q + kvh * G + qi) * max_splits + slot;
      part_o[pidx * HD + d] = oo;
      if (d == 0) {
        part_ml[pidx * 2] = mm;
        part_ml[pidx * 2 + 1] = ll;
      }
    }
    __syncthreads();  // s_o / s_ml are rewritten by the next item
  }
}

// Split merge: one wave per (row, query head), four per workgroup.  Lane s holds split s's
// (m, l) -- all of them fetched by ONE load instruction, reduced with cross-lane ops --
// then every split's O partial (HD floats, one coalesced load per split, HD / 64 per lane)
// is weighted by its factor, broadcast with v_readlane.  The former one-thread-per-dim
// form walked the splits with dependent broadcast loads twice (35 us per layer at B = 616).
constexpr int COMBINE_WAVES = 4;
template <int HD>
__global__ __launch_bounds__(64 * COMBINE_WAVES) void decode_combine_kernel(
    const float* __restrict__ part_o, const float* __restrict__ part_ml, const int* __restrict__ seq_lens, int n_q,
    int max_splits, int split_tokens, int n_bq, bf16_t* __restrict__ out, const int* __restrict__ kv_begin,
    const int* __restrict__ split_base) {
  constexpr int PER = HD / 64;  // dims per lane
  const int lane = threadIdx.x & 63;
  const int bq = blockIdx.x * COMBINE_WAVES + (threadIdx.x >> 6);
  if (bq >= n_bq) return;  // wave-uniform
  const int b = bq / n_q;
  const int own = max(0, seq_lens[b] - (kv_begin ? kv_begin[b] : 0));
  // <= max_splits <= 64 (host check); slots 0 .. split_base[b]-1 hold the shared-prefix partials
  const int ns = (split_base ? split_base[b] : 0) + (own + split_tokens - 1) / split_tokens;
  const float2 mlv = lane < ns ? reinterpret_cast<const float2*>(part_ml)[static_cast<size_t>(bq) * max_splits + lane]
                               : float2{-INFINITY, 0.f};
  float mm = mlv.x;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) mm = fmaxf(mm, __shfl_xor(mm, o, 64));
  const float f = mlv.x == -INFINITY ? 0.f : exp2f(mlv.x - mm);
  float ll = mlv.y * f;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) ll += __shfl_xor(ll, o, 64);
  const float* po = part_o + static_cast<size_t>(bq) * max_splits * HD + lane * PER;
  float acc[PER];
#pragma unroll
  for (int e = 0; e < PER; ++e) acc[e] = 0.f;
  int s = 0;
  for (; s + 4 <= ns; s += 4) {  // four splits' loads in flight before their FMAs
    float v[4][PER];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < PER; ++e) v[j][e] = po[(s + j) * HD + e];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float fj = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, f), s + j));
#pragma unroll
      for (int e = 0; e < PER; ++e) acc[e] += fj * v[j][e];
    }
  }
  for (; s < ns; ++s) {
    const float fj = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, f), s));
#pragma unroll
    for (int e = 0; e < PER; ++e) acc[e] += fj * po[s * HD + e];
  }
  const float inv = ll > 0.f ? 1.f / ll : 0.f;
#pragma unroll
  for (int e = 0; e < PER; ++e) out[static_cast<size_t>(bq) * HD + lane * PER + e] = f2bf(acc[e] * inv);
}

// ------------------------------------------------------- decode, shared prefix
// Work item (one wave) = (group, 64-column block, shared split) for the kv head blockIdx.y.  A group's
// columns are its (member, query head) pairs, c = member * G + head, 16 per MFMA tile and
// SH_NT tiles per wave, so the G = n_q / n_kv heads of up to 64 / G rows share every
// 16-B K/V load (the per-row kernel packs only one row's G heads into the 16 columns).
// grp_desc[grp] = {first member in grp_rows, members, shared blocks, unused}; the shared
// block ids are read from the first member's table row (every member holds the same ids
// there).  The shared tokens are all visible to every member (they precede each member's
// own tokens), so the loop is the prefill kernel's full-visibility block (K/V reloaded in
// place, lazy rescale outside the inner loop) plus one masked half chunk for an odd block
// count.  Splitting the shared tokens into split_tokens pieces (own slots) keeps each wave's
// dependent chunk chain short: one whole-prefix item per wave was latency-bound (a 640-token
// prefix = 20 chained chunk loads) and left most SIMDs idle.  Out: slot `split` of each
// member's (m, l, O) partials.  Every table entry is
// range-checked before use: a bad item is skipped, never dereferenced.
constexpr int SH_NT = 4;
constexpr int SH_WAVES = 4;

template <int HD, bool F8>
__global__ __launch_bounds__(64 * SH_WAVES) void decode_shared_kernel(
    const bf16_t* __restrict__ q, KVGeom g, const int* __restrict__ block_tables, int max_blocks, int B, int n_q,
    float scale_log2, const int* __restrict__ grp_rows, int grp_cap, const int* __restrict__ grp_desc,
    int max_groups, const int* __restrict__ items, const int* __restrict__ n_items_p, int max_items,
    int split_tokens, float* __restrict__ part_o, float* __restrict__ part_ml, int max_splits) {
  constexpr int NT = SH_NT;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, h = lane >> 4;
  const int kvh = blockIdx.y;
  const int G = n_q / g.n_kv;
  const int n_items = min(*n_items_p, max_items);
  for (int it = blockIdx.x * SH_WAVES + w; it < n_items; it += gridDim.x * SH_WAVES) {
    const int grp = items[4 * it], cb = items[4 * it + 1], sp = items[4 * it + 2];
    if (grp < 0 || grp >= max_groups || cb < 0 || sp < 0 || sp >= max_splits) continue;  // wave-uniform
    const int mbeg = grp_desc[4 * grp], nmem = grp_desc[4 * grp + 1], nblk = grp_desc[4 * grp + 2];
    if (mbeg < 0 || nmem <= 0 || mbeg + nmem > grp_cap || nblk <= 0 || nblk > max_blocks) continue;
    const int lead = grp_rows[mbeg];
    if (lead < 0 || lead >= B) continue;
    const int* table = block_tables + static_cast<size_t>(lead) * max_blocks;
    const int S = nblk * BS;
    const int t_lo = sp * split_tokens, t_hi = min(S, t_lo + split_tokens);  // this item's shared tokens
    if (t_lo >= S) continue;
    const int ncol = nmem * G;

    bf16x8 bq[NT][HD / 32];
    int qrow[NT], qhd[NT];  // this lane's column: row and query head (qrow < 0: no column)
    float m[NT], l[NT];
    f32x4 o[NT][HD / 16];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int col = cb * (16 * NT) + nt * 16 + r;
      const int mem = col / G;
      int row = col < ncol ? grp_rows[mbeg + mem] : -1;
      if (row >= B) row = -1;
      const int hq = kvh * G + (col - mem * G);
      load_q<HD>(bq[nt], q + (static_cast<size_t>(row >= 0 ? row : 0) * n_q + (row >= 0 ? hq : 0)) * HD, row >= 0,
                 lane);
      qrow[nt] = row;
      qhd[nt] = hq;
      m[nt] = -INFINITY;
      l[nt] = 0.f;
#pragma unroll
      for (int dt = 0; dt < HD / 16; ++dt) o[nt][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

    // absolute chunk indices; split_tokens is a multiple of CHUNK, so only the group's last
    // split can end in a half chunk (odd block count)
    const int nchunk = (t_hi + CHUNK - 1) / CHUNK, n_full = t_hi / CHUNK;
    int c = t_lo / CHUNK;
    Chunk<HD, F8> cur;
    load_chunk<HD, F8>(cur, g, table[2 * c], table[min(2 * c + 1, nblk - 1)], kvh, lane);
    while (c < n_full) {
      f32x2 t[NT][4];
      float mx[NT];
      bool grow = false;
      int b0 = 0, b1 = 0;
      for (; c < n_full; ++c) {
        const int cn = min(c + 1, nchunk - 1);
        b0 = table[2 * cn], b1 = table[min(2 * cn + 1, nblk - 1)];
        grow = full_scores<HD, NT, F8>(cur, bq, scale_log2, m, t, mx,
                                       [&](Chunk<HD, F8>& x) { load_chunk_k<HD, F8>(x, g, b0, b1, kvh, lane); });
        if (grow) break;  // wave-uniform
        full_pv<HD, NT, F8>(cur, t, l, o,
                            [&](Chunk<HD, F8>& x) { load_chunk_v<HD, F8>(x, g, b0, b1, kvh, lane); });
      }
      if (!grow) break;
      full_rescale<HD, NT>(mx, m, l, o, t);
      full_pv<HD, NT, F8>(cur, t, l, o,
                          [&](Chunk<HD, F8>& x) { load_chunk_v<HD, F8>(x, g, b0, b1, kvh, lane); });
      ++c;
    }
    if (c < nchunk) {  // odd block count: the last 16 tokens, masked at S (cur holds that chunk)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        compute_chunk<HD, AllVisible, true, F8>(cur, bq[nt], c * CHUNK, t_hi, AllVisible{}, scale_log2, m[nt],
                                                l[nt], o[nt], lane);
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      if (qrow[nt] < 0) continue;
      const size_t pidx = (static_cast<size_t>(qrow[nt]) * n_q + qhd[nt]) * max_splits + sp;
#pragma unroll
      for (int dt = 0; dt < HD / 16; ++dt)
        *reinterpret_cast<f32x4*>(part_o + pidx * HD + dt * 16 + 4 * h) = o[nt][dt];
      if (h == 0) {
        part_ml[pidx * 2] = m[nt];
        part_ml[pidx * 2 + 1] = l[nt];
      }
    }
  }
}

struct Cascade {
  const int* kv_begin;    // [B] shared tokens per row (0: none)
  const int* split_base;  // [B] shared-pass splits of the row (its partial slots 0 .. split_base-1)
  const int* grp_rows;    // [grp_cap] members, grouped
  int grp_cap;
  const int* grp_desc;    // [max_groups, 4]
  int max_groups;
  const int* items;       // [max_items, 4] (group, 64-column block, shared split, -)
  const int* n_items;     // [1] live items (device: graph replays see the current count)
  int max_items;
  int split_tokens;       // shared tokens per item (a multiple of CHUNK)
};

template <int HD, bool F8 = false, int CPW = 1>
void launch_decode(const bf16_t* q, KVGeom g, const int* tables, int max_blocks, const int* seq_lens, int B,
                   int n_q, float sl, float* ws, int max_splits, bf16_t* out, const Cascade& cas,
                   hipStream_t stream) {
  constexpr int DEC_SPLIT = DEC_WAVES * CHUNK * CPW;
  float* part_o = ws;
  float* part_ml = ws + static_cast<size_t>(B) * n_q * max_splits * HD;
  if (cas.kv_begin != nullptr && cas.max_items > 0) {
    // grid fixed by the item capacity (graph-safe); the live count is read on the device
    const int per_kv = std::max(1, std::min((cas.max_items + SH_WAVES - 1) / SH_WAVES, 128));
    hipLaunchKernelGGL((decode_shared_kernel<HD, F8>), dim3(per_kv, g.n_kv), dim3(64 * SH_WAVES), 0, stream, q, g,
                       tables, max_blocks, B, n_q, sl, cas.grp_rows, cas.grp_cap, cas.grp_desc, cas.max_groups,
                       cas.items, cas.n_items, cas.max_items, cas.split_tokens, part_o, part_ml, max_splits);
  }
  // fixed (graph-safe) grid striding over the live items: one full wave of resident workgroups
  static int resident = 0;
  if (resident == 0) {
    int per_cu = 0, cus = 0, dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, decode_attn_kernel<HD, F8, CPW>, 256, 0);
    resident = std::max(1, per_cu) * std::max(1, cus);
  }
  const int grid = static_cast<int>(std::min<long>(static_cast<long>(B) * g.n_kv * max_splits, resident));
  hipLaunchKernelGGL((decode_attn_kernel<HD, F8, CPW>), dim3(grid), dim3(256), 0, stream, q, g, tables, max_blocks,
                     seq_lens, B, n_q, sl, part_o, part_ml, max_splits, cas.kv_begin, cas.split_base);
  const int n_bq = B * n_q;
  hipLaunchKernelGGL(decode_combine_kernel<HD>, dim3((n_bq + COMBINE_WAVES - 1) / COMBINE_WAVES),
                     dim3(64 * COMBINE_WAVES), 0, stream, part_o, part_ml, seq_lens, n_q, max_splits, DEC_SPLIT, n_bq,
                     out, cas.kv_begin, cas.split_base);
}

// ----------------------------------------------------------------- prefill
// tiles[i] = {b, q_begin, q_end} (packed row indices); q rows of sequence b occupy
// [q_start[b], q_start[b+1]) and are its last rows (positions ctx-qlen .. ctx-1).
//
// A workgroup = 4 waves over one 64-row tile.  Each wave owns NT column tiles
// of 16 query rows (16*NT rows) of ONE query head and streams the kv head's
// K/V once for all of them: every 16-B K/V load feeds NT times the MFMAs of
// the one-tile (NT = 1) form, which was load-bound (L2 -> CU) at 120-200 TF/s.
// Waves of a block: 4/NT row groups x NT heads; grid = (tiles, ceil(n_q/NT)).
#ifndef PREFILL_LAZY
#define PREFILL_LAZY false  // measured: see PERF.md (lazy spills at NT = 4)
#endif
#ifndef PREFILL_FULL_BLOCK
#define PREFILL_FULL_BLOCK 1  // fully visible chunks through full_scores / full_pv (lazy rescale outside the inner loop, in-place reload)
#endif
#ifndef PREFILL_LDS_BUILD
#define PREFILL_LDS_BUILD 0  // compile the shared K/V ring form (LDSKV) into this library
#endif
#ifndef PREFILL_LDS
#define PREFILL_LDS 0  // with PREFILL_LDS_BUILD: use the ring by default; BCG_PREFILL_LDS=0/1 overrides at run time
#endif
#ifndef PREFILL_XCD_ORDER
#define PREFILL_XCD_ORDER 0  // default grid order (BCG_PREFILL_XCD_ORDER=0/1 overrides at run time)
#endif
#ifndef PREFILL_WPE
#define PREFILL_WPE 0
#endif
#if PREFILL_WPE
#define PREFILL_ATTR __attribute__((amdgpu_waves_per_eu(PREFILL_WPE, PREFILL_WPE)))
#else
#define PREFILL_ATTR
#endif
// LDSKV (bf16 cache, HD = 128, NT = 4): the 4 waves of a workgroup are 4 consecutive query heads
// (at most 2 kv heads when G >= 2); each 32-token chunk of both kv heads' K and V goes global -> LDS
// ONCE per workgroup by LDS-DMA (8 x 1-KiB pieces per wave), 4-slot ring, issued 2 chunks ahead;
// the in-place reloads of the full-visibility loop then read their fragments from LDS
// (XOR-swizzled K rows: conflict-free ds_read_b128) instead of issuing 16 global loads per wave.
// One raw s_barrier per chunk (all waves share the rows, so they run the same chunks).
__device__ __forceinline__ int kswz(int row) { return ((row & 3) | ((row & 8) >> 1)) << 1; }

template <int HD, int NT, bool F8 = false, bool LDSKV = false>
__global__ __launch_bounds__(256) PREFILL_ATTR void prefill_attn_kernel(
    const bf16_t* __restrict__ q, KVGeom g, const int* __restrict__ block_tables, int max_blocks,
    const int* __restrict__ q_start, const int* __restrict__ seq_lens, const int* __restrict__ tiles,
    int n_q, float scale_log2, bf16_t* __restrict__ out, int n_tiles, int xcd_order) {
  constexpr int RG = 4 / NT;   // row groups per 64-row tile
  constexpr int ROWS = 16 * NT;
  // xcd_order: 1-D grid; workgroup id b runs on XCD b % 8 (round-robin dispatch), so the
  // head groups of one tile are given consecutive ids of ONE XCD -- the query heads that share
  // a kv head then read its K/V through that XCD's L2 together -- while each XCD still walks
  // the tiles in the host's deepest-first order (tile = 8 * local index + XCD).
  int tile, hgrp;
  if (xcd_order) {
    const int hg_n = (n_q + NT - 1) / NT, s = blockIdx.x >> 3;
    tile = (s / hg_n) * 8 + (blockIdx.x & 7);
    hgrp = s % hg_n;
    if (tile >= n_tiles) return;  // padding of the grid to whole XCD rounds
  } else {
    tile = blockIdx.x;
    hgrp = blockIdx.y;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int qh = hgrp * NT + w / RG;
  if (qh >= n_q) return;  // wave-uniform; no block-level barriers in this kernel
  const int b = tiles[3 * tile], q_begin = tiles[3 * tile + 1], q_end = tiles[3 * tile + 2];
  const int r = lane & 15, h = lane >> 4;
  const int row0 = q_begin + ROWS * (w % RG);
  if (row0 >= q_end) return;
  const int ctx = seq_lens[b];
  const int qs = q_start[b], qlen = q_start[b + 1] - qs;
  const int pos0 = ctx - qlen;  // position of row qs
  const int kvh = qh / (n_q / g.n_kv);
  const int* table = block_tables + static_cast<size_t>(b) * max_blocks;

  bf16x8 bq[NT][HD / 32];
  float m[NT], l[NT];
  f32x4 o[NT][HD / 16];
  // query position of this lane's column; per sub-tile: first row's position, exclusive key bound
  int my_pos[NT], sub_first[NT], sub_end[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int my_row = row0 + 16 * nt + r;
    const bool ok = my_row < q_end;
    load_q<HD>(bq[nt], q + (static_cast<size_t>(ok ? my_row : row0) * n_q + qh) * HD, ok, lane);
    my_pos[nt] = pos0 + (my_row - qs);
    sub_first[nt] = pos0 + (row0 + 16 * nt - qs);
    sub_end[nt] = pos0 + (min(row0 + 16 * nt + 15, q_end - 1) - qs) + 1;
    m[nt] = -INFINITY;
    l[nt] = 0.f;
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) o[nt][dt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int last_row = min(row0 + ROWS - 1, q_end - 1);
  const int kv_end = pos0 + (last_row - qs) + 1;  // exclusive bound of keys visible to this wave

  // block ids in windows of 64 (one per lane), broadcast with readlane (see decode)
  const int nblk = (kv_end + BS - 1) / BS;
  int win_base = 0;
  int my_blk = lane < nblk ? table[lane] : 0;
  auto block_at = [&](int bi) -> int {
    if (bi >= win_base + 64) {  // wave-uniform: advance the window
      win_base += 64;
      my_blk = win_base + lane < nblk ? table[win_base + lane] : 0;
    }
    return __builtin_amdgcn_readlane(my_blk, bi - win_base);
  };
  // next-chunk loads issued unconditionally (clamped to the last chunk) -- see decode
  const int nchunk = (kv_end + CHUNK - 1) / CHUNK;
  Chunk<HD, F8> cur;
  load_chunk<HD, F8>(cur, g, block_at(0), block_at(min(1, nblk - 1)), kvh, lane);
#if PREFILL_FULL_BLOCK
  // chunks every row of the wave sees in full: one interleaved block for all NT sub-tiles,
  // the next chunk reloaded in place (K after the S^T MFMAs, V after the P.V MFMAs): no
  // second register set for the prefetch
  int c = 0;
  const int n_full = min(sub_first[0] / CHUNK, nchunk);  // chunks every row of the wave sees in full

  // ---- LDSKV: shared K/V ring (see above the kernel) ----
  constexpr int KV_SLOTS = 4, KV_HALF = 8192, KV_HEAD = 2 * KV_HALF, KV_SLOT = 2 * KV_HEAD;
  __shared__ __attribute__((aligned(1024))) unsigned char kv_ring[LDSKV ? KV_SLOTS * KV_SLOT : 16];
  const int kvA = LDSKV ? (hgrp * NT) / (n_q / g.n_kv) : 0;
  const int kvsel = kvh - kvA;                                              // which staged kv head this wave reads
  const int dkv = min(kvA + (w >> 1), (hgrp * NT + NT - 1) / (n_q / g.n_kv));  // kv head this wave stages
  // block ids of the DMA lookahead: scalar loads (lgkmcnt) -- a vector load here would make every
  // wait on it (vmcnt counts in order) drain the DMA pieces in flight ahead of it
  auto block_at2 = [&](int bi) -> int { return table[__builtin_amdgcn_readfirstlane(bi)]; };
  auto issue_chunk = [&](int k) {  // this wave's 8 pieces (K or V of kv head dkv) of chunk k
    if constexpr (LDSKV && !F8) {
      const int bb0 = block_at2(2 * k), bb1 = block_at2(min(2 * k + 1, nblk - 1));
      unsigned char* dst = kv_ring + (k % KV_SLOTS) * KV_SLOT + (w >> 1) * KV_HEAD + (w & 1) * KV_HALF;
      const unsigned char* kc = reinterpret_cast<const unsigned char*>(g.k);
      const unsigned char* vc = reinterpret_cast<const unsigned char*>(g.v);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const size_t base = 2 * block_base<HD>(g, i < 4 ? bb0 : bb1, dkv);
        const unsigned char* src;
        if ((w & 1) == 0) {  // K rows (i & 3) * 4 + lane / 16; the lane's LDS slot p holds chunk p ^ kswz(row)
          const int row = (i & 3) * 4 + (lane >> 4);
          src = kc + base + row * 256 + ((lane & 15) ^ kswz(row)) * 16;
        } else {  // V^T: a plain copy of the block-head's 4 KiB
          src = vc + base + (i & 3) * 1024 + lane * 16;
        }
        __builtin_amdgcn_global_load_lds(src, dst + i * 1024, 16, 0, 0);
      }
    }
  };
  auto lds_k = [&](Chunk<HD, F8>& x, int k) {
    if constexpr (LDSKV && !F8) {
      const unsigned char* base = kv_ring + (k % KV_SLOTS) * KV_SLOT + kvsel * KV_HEAD;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int t = 8 * (r >> 2) + 4 * u + (r & 3), row = t & 15;
#pragma unroll
        for (int kk = 0; kk < HD / 32; ++kk)
          x.k[u][kk] =
              *reinterpret_cast<const bf16x8*>(base + (t >> 4) * 4096 + row * 256 + ((4 * kk + h) ^ kswz(row)) * 16);
      }
    }
  };
  auto lds_v = [&](Chunk<HD, F8>& x, int k) {
    if constexpr (LDSKV && !F8) {
      const unsigned char* base =
          kv_ring + (k % KV_SLOTS) * KV_SLOT + kvsel * KV_HEAD + KV_HALF + (h >> 1) * 4096 + (h & 1) * 16;
#pragma unroll
      for (int dt = 0; dt < HD / 16; ++dt) x.v[dt] = *reinterpret_cast<const bf16x8*>(base + (dt * 16 + r) * 32);
    }
  };
  if constexpr (LDSKV && !F8) {  // chunks 1 and 2 ahead of the loop; chunk k + 3 is issued in iteration k
    if (1 < min(n_full + 1, nchunk)) issue_chunk(1);
    if (2 < min(n_full + 1, nchunk)) issue_chunk(2);
  }
  // LDSKV: chunks 1 .. n_stage-1 go through the ring -- every full chunk's successor, including
  // the first masked chunk, which the masked loop below then starts from
  const int n_stage = min(n_full + 1, nchunk);
  auto ring_k = [&](Chunk<HD, F8>& x) {
    if (c + 1 >= n_stage) return;  // no successor (the wave's last chunk): nothing to reload
    // this wave's pieces of chunk c+1 landed (chunk c+2's 8 may still fly), then every wave's
    if (c + 2 < n_stage) {
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();  // ... and every wave is past chunk c-1: its slot is free
    asm volatile("" ::: "memory");
    if (c + 3 < n_stage) issue_chunk(c + 3);
    lds_k(x, c + 1);
  };
  auto ring_v = [&](Chunk<HD, F8>& x) {
    if (c + 1 < n_stage) lds_v(x, c + 1);
  };
  if constexpr (LDSKV && !F8) {
    // no VGPR-destination global load in this loop: with one, the compiler's wait before the
    // S^T MFMAs would be a vmcnt(0) that drains the ring every chunk
    while (c < n_full) {
      f32x2 t[NT][4];
      float mx[NT];
      bool grow = false;
      for (; c < n_full; ++c) {
        grow = full_scores<HD, NT, F8>(cur, bq, scale_log2, m, t, mx, ring_k);
        if (grow) break;  // wave-uniform
        full_pv<HD, NT, F8>(cur, t, l, o, ring_v);
      }
      if (!grow) break;
      full_rescale<HD, NT>(mx, m, l, o, t);
      full_pv<HD, NT, F8>(cur, t, l, o, ring_v);
      ++c;
    }
  } else {
    while (c < n_full) {
      f32x2 t[NT][4];
      float mx[NT];
      bool grow = false;
      int b0 = 0, b1 = 0;
      // inner loop: no VALU on O (it stays in the MFMA accumulators); leaves with S live
      // when a column's max moved enough to need the lazy rescale
      for (; c < n_full; ++c) {
        const int cn = min(c + 1, nchunk - 1);
#ifdef PREFILL_ABL_HOT  // timing ablation only (wrong results): every reload re-reads chunk 0's blocks (L2-hot)
        b0 = block_at(0), b1 = block_at(min(1, nblk - 1));
#else
        b0 = block_at(2 * cn), b1 = block_at(min(2 * cn + 1, nblk - 1));
#endif
        grow = full_scores<HD, NT, F8>(cur, bq, scale_log2, m, t, mx,
                                       [&](Chunk<HD, F8>& x) { load_chunk_k<HD, F8>(x, g, b0, b1, kvh, lane); });
        if (grow) break;  // wave-uniform
        full_pv<HD, NT, F8>(cur, t, l, o,
                            [&](Chunk<HD, F8>& x) { load_chunk_v<HD, F8>(x, g, b0, b1, kvh, lane); });
      }
      if (!grow) break;
      full_rescale<HD, NT>(mx, m, l, o, t);
      full_pv<HD, NT, F8>(cur, t, l, o,
                          [&](Chunk<HD, F8>& x) { load_chunk_v<HD, F8>(x, g, b0, b1, kvh, lane); });
      ++c;
    }
  }
  Chunk<HD, F8> nxt;
  for (; c < nchunk; ++c) {
#else
  Chunk<HD, F8> nxt;
  for (int c = 0; c < nchunk; ++c) {
#endif
    const int cn = min(c + 1, nchunk - 1);
    load_chunk<HD, F8>(nxt, g, block_at(2 * cn), block_at(min(2 * cn + 1, nblk - 1)), kvh, lane);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      if (c * CHUNK >= sub_end[nt]) continue;  // wave-uniform: chunk wholly in this sub-tile's causal future
      if ((c + 1) * CHUNK <= sub_first[nt])     // wave-uniform: every key visible to every row
        compute_chunk<HD, Causal, false, F8, PREFILL_LAZY>(cur, bq[nt], c * CHUNK, sub_end[nt], Causal{my_pos[nt]},
                                                           scale_log2, m[nt], l[nt], o[nt], lane);
      else
        compute_chunk<HD, Causal, true, F8, PREFILL_LAZY>(cur, bq[nt], c * CHUNK, sub_end[nt], Causal{my_pos[nt]},
                                                          scale_log2, m[nt], l[nt], o[nt], lane);
    }
    cur = nxt;
  }
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int my_row = row0 + 16 * nt + r;
    if (my_row >= q_end) continue;
    const float inv = l[nt] > 0.f ? 1.f / l[nt] : 0.f;
    bf16_t* orow = out + (static_cast<size_t>(my_row) * n_q + qh) * HD;
    // O^T rows d = 16dt + 4h + i are this lane's column (query my_row)
#pragma unroll
    for (int dt = 0; dt < HD / 16; ++dt) {
      u16x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = f2bf(o[nt][dt][i] * inv);
      *reinterpret_cast<u16x4*>(orow + dt * 16 + 4 * h) = v;
    }
  }
}

template <int HD, bool F8>
void launch_prefill(int n_tiles, int n_q, const bf16_t* q, KVGeom g, const int* tables, int max_blocks,
                    const int* q_start, const int* seq_lens, const int* tiles, float sl, bf16_t* out,
                    hipStream_t stream) {
#ifndef PREFILL_NT
#define PREFILL_NT 4
#endif
  constexpr int NT = PREFILL_NT;  // 1 and 2 measured slower (PERF.md); the LDS-shared forms were 180-200 TF/s
  const int hg_n = (n_q + NT - 1) / NT;
  static const int xcd_order = [] {
    const char* e = std::getenv("BCG_PREFILL_XCD_ORDER");
    return e ? std::atoi(e) : PREFILL_XCD_ORDER;
  }();
  static const int lds_env = [] {
    const char* e = std::getenv("BCG_PREFILL_LDS");
    return e ? std::atoi(e) : PREFILL_LDS;
  }();
  // the shared K/V ring needs whole 4-head workgroups spanning <= 2 kv heads, HD = 128, bf16 KV
  const bool lds = lds_env && HD == 128 && !F8 && NT == 4 && n_q % 4 == 0 && n_q / g.n_kv >= 2;
  const dim3 grid = xcd_order ? dim3(((n_tiles + 7) / 8) * 8 * hg_n) : dim3(n_tiles, hg_n);
#if PREFILL_LDS_BUILD  // the shared-ring form lost its A/B: only variant builds carry it (-DPREFILL_LDS_BUILD=1)
  if (lds) {
    hipLaunchKernelGGL((prefill_attn_kernel<HD, NT, F8, true>), grid, dim3(256), 0, stream, q, g, tables, max_blocks,
                       q_start, seq_lens, tiles, n_q, sl, out, n_tiles, xcd_order);
    return;
  }
#else
  (void)lds;
#endif
  hipLaunchKernelGGL((prefill_attn_kernel<HD, NT, F8, false>), grid, dim3(256), 0, stream, q, g, tables, max_blocks,
                     q_start, seq_lens, tiles, n_q, sl, out, n_tiles, xcd_order);
}

// ------------------------------------------------- prefill, 32x32 MFMA, LDS-staged K/V
// The 16x16 kernel above holds 510 registers (one wave per SIMD), so nothing hides a wave's
// softmax VALU or its reload latency behind another wave's MFMAs.  This form is built for two
// waves per SIMD (<= 256 registers): a workgroup = NW waves x 32 query rows of ONE query head
// (tiles of 32 * NW rows), K/V of 64-token chunks staged ONCE per workgroup in an NS-slot LDS
// ring by LDS-DMA (32 x 1-KiB pieces per chunk, P = 32 / NW per wave), one s_barrier per chunk.
//
// Swapped products on v_mfma_f32_32x32x16_bf16 (A[m = l&31][k = 8(l>>5)+j], B[k][n = l&31],
// C[m = 8(i>>2) + 4(l>>5) + (i&3)][n = l&31]):
//   S^T = K Q^T     A = K rows from LDS, B = Q fragments in registers (8 x bf16x8);
//   O^T += V^T P^T  A = V^T rows from LDS (the V cache is [hd][16 tokens] per block),
//                   B = P^T straight from the S^T accumulators of the same lane.
// Token permutation (per 32-token tile u): S^T row m = 16s + 8a + 4h + b holds token
// 32u + 16s + 8h + 4a + b, so accumulator i of lane half h is token 32u + 16(i>>3) + 8h + (i&7):
// P.V k-step 2u + (i>>3) takes the lane's own 8 consecutive accumulators as its B operand, and
// the matching V^T operand is ONE 16-byte read (8 consecutive tokens of a V^T row).  No
// cross-lane traffic except one permlane32_swap per chunk for the column max.
// LDS images (no bank conflicts for the 16-lane groups of ds_read_b128):
//   K: row t (token of the chunk) at t * 256, its 16-B chunk p stored at slot p ^ (t & 15);
//   V: block s at 16 KiB + s * 4 KiB, row d at d * 32, 16-B half e stored at e ^ ((d >> 3) & 1).
// The source side of each LDS-DMA lane applies the swizzle (LDS destinations are consecutive).
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int PREFILL32_MAX_BLOCKS = 1024;  // block-table width the 32x32 kernel stages in LDS (16k tokens)

// One 64-token chunk of prefill_attn32_kernel for one wave (32 query columns):
//   attn32_scores  S^T = K Q^T, the column max m_new (the online softmax rescales EVERY chunk:
//                  a data-dependent rescale branch made hipcc copy the 64 O accumulators between
//                  register sets on every chunk -- 64 v_mov_b64 against 32 v_pk_mul here),
//                  O and the partial sums scaled by 2^(m - m_new), t = S * scale - m_new;
//   attn32_pv      P = 2^t, partial row sums, O^T += V^T P^T.
// MASKED: rel_pos = (token of accumulator 0) - (this column's position) (causal mask),
// rel_ctx = (token of accumulator 0) - ctx (V of tokens past the context is zeroed).
// A column's first chunk always holds a visible key (token 0), so m is finite after it.
template <bool MASKED>
__device__ __forceinline__ void attn32_scores(const unsigned char* slot, int k_lane, const bf16x8 (&bq)[8],
                                              float scale_log2, int rel_pos, float& m, float& lsum,
                                              f32x16 (&o)[4], float (&t)[32]) {
  f32x16 s0 = f32x16{}, s1 = f32x16{};
  bf16x8 ka[8][2];
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    const unsigned char* p = slot + (k_lane ^ (kk << 5));
    ka[kk][0] = *reinterpret_cast<const bf16x8*>(p);
    ka[kk][1] = *reinterpret_cast<const bf16x8*>(p + 32 * 256);
  }
  __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead (the scheduler sinks them to their uses)
#pragma unroll
  for (int kk = 0; kk < 8; ++kk) {
    s0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka[kk][0], bq[kk], s0, 0, 0, 0);
    s1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ka[kk][1], bq[kk], s1, 0, 0, 0);
  }
  // accumulator i of tile u is token 32u + 16(i>>3) + 8h + (i&7)
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    t[i] = s0[i];
    t[16 + i] = s1[i];
  }
  if constexpr (MASKED) {
#pragma unroll
    for (int i = 0; i < 32; ++i)
      if (rel_pos + 32 * (i >> 4) + 16 * ((i >> 3) & 1) + (i & 7) > 0) t[i] = -INFINITY;
  }
  float v = t[0];
#pragma unroll
  for (int i = 1; i < 31; i += 2) v = vmax3(v, t[i], t[i + 1]);
  v = vmax(v, t[31]);
  const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = vmax(__uint_as_float(sw[0]), __uint_as_float(sw[1])) * scale_log2;  // column max (log2 units)
  const float m_new = vmax(m, v);   // finite from the column's first chunk on
  const float alpha = fast_exp2(m - m_new);  // m = -inf: 0
  m = m_new;
  lsum *= alpha;
  const f32x2 al = {alpha, alpha};
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
      const f32x2 x = f32x2{o[dt][i], o[dt][i + 1]} * al;
      o[dt][i] = x.x;
      o[dt][i + 1] = x.y;
    }
  const f32x2 sc = {scale_log2, scale_log2}, mm = {m_new, m_new};
#pragma unroll
  for (int i = 0; i < 32; i += 2) {  // two scores per v_pk_fma_f32 (masked: -inf stays -inf)
    const f32x2 x = f32x2{t[i], t[i + 1]} * sc - mm;
    t[i] = x.x;
    t[i + 1] = x.y;
  }
}

template <bool MASKED>
__device__ __forceinline__ void attn32_pv(const unsigned char* slot, int v_lane, int rel_ctx, const float (&t)[32],
                                          float& lsum, f32x16 (&o)[4]) {
  // P = 2^t, lane-local partial row sums (packed adds); P^T operands of the four 16-token k-steps
  bf16x8 bp[4];
  f32x2 ps = {0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 32; i += 2) {
    const f32x2 p = {fast_exp2(t[i]), fast_exp2(t[i + 1])};
    ps += p;
    bp[i >> 3][i & 7] = static_cast<__bf16>(p.x);
    bp[i >> 3][(i & 7) + 1] = static_cast<__bf16>(p.y);
  }
  lsum += ps.x + ps.y;
  // O^T += V^T P^T (k-step s = block s of the chunk, this lane half's 8 tokens); each V operand
  // is read one MFMA ahead
  const unsigned char* vb = slot + v_lane;
  u32x4 va = *reinterpret_cast<const u32x4*>(vb);
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    uint32_t keep[4] = {~0u, ~0u, ~0u, ~0u};
    if constexpr (MASKED) {  // stale bytes past the context may be non-finite: zero them
#pragma unroll
      for (int j2 = 0; j2 < 4; ++j2) {
        const int tk = rel_ctx + 16 * s + 2 * j2;  // token - ctx
        keep[j2] = (tk < 0 ? 0x0000ffffu : 0u) | (tk + 1 < 0 ? 0xffff0000u : 0u);
      }
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const int nx = 4 * s + dt + 1;
      u32x4 vn = va;
      if (nx < 16) vn = *reinterpret_cast<const u32x4*>(vb + (nx >> 2) * 4096 + (nx & 3) * 1024);
      if constexpr (MASKED) {
#pragma unroll
        for (int j2 = 0; j2 < 4; ++j2) va[j2] &= keep[j2];
      }
      o[dt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, va), bp[s], o[dt], 0, 0, 0);
      va = vn;
    }
  }
}

template <int NW, int NS>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(2))) void prefill_attn32_kernel(
    const bf16_t* __restrict__ q, KVGeom g, const int* __restrict__ block_tables, int max_blocks,
    const int* __restrict__ q_start, const int* __restrict__ seq_lens, const int* __restrict__ tiles, int n_q,
    float scale_log2, bf16_t* __restrict__ out, int n_tiles) {
  constexpr int HD = 128, KC = 64;                   // head dim, tokens per chunk
  constexpr int KBYTES = KC * HD * 2, SLOT = 2 * KBYTES;  // K (then V) image of one chunk: 16 KiB each
  constexpr int P = 32 / NW;                         // 1-KiB DMA pieces per wave per chunk
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  static_assert(NS >= 2 && NS <= 4, "ring depth");
  __shared__ __attribute__((aligned(1024))) unsigned char ring[NS * SLOT];

  // XCD-grouped order (1-D grid): workgroup id i runs on XCD i % 8, so kv head i % n_kv puts every
  // query head of a kv head on the same XCD(s) (one XCD per kv head at n_kv = 8), the G heads of
  // one tile next to each other: the K/V chunks they all stage come from that XCD's L2 (+5-8 %
  // over a (tile, head) grid, profiles/r6_prefill32)
  const int G = n_q / g.n_kv;
  const int kvh = blockIdx.x % g.n_kv, rest = blockIdx.x / g.n_kv;
  const int tile = rest / G, qh = kvh * G + rest % G;
  if (tile >= n_tiles) return;
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int col = lane & 31, h = lane >> 5;
  const int b = tiles[3 * tile], q_begin = tiles[3 * tile + 1], q_end = tiles[3 * tile + 2];
  const int ctx = seq_lens[b];
  const int pos0 = ctx - (q_start[b + 1] - q_start[b]) - q_start[b];  // position of packed row r = pos0 + r
  const int* table = block_tables + static_cast<size_t>(b) * max_blocks;
  const int nblk = (ctx + BS - 1) / BS;
  const int wg_last = min(q_begin + 32 * NW, q_end) - 1;
  const int nchunk = (pos0 + wg_last + KC) / KC;      // chunks the workgroup stages (uniform)
  const int row0 = q_begin + 32 * w;
  const bool active = row0 < q_end;                   // wave-uniform
  const int w_last = min(row0 + 31, q_end - 1);
  const int w_chunks = active ? (pos0 + w_last + KC) / KC : 0;          // chunks this wave computes
  const int n_full = active ? min((pos0 + row0 + 1) / KC, w_chunks) : 0;  // ... seen in full by all its rows
  // this lane's query column; columns past q_end compute as the tile's last row (never stored)
  const int my_row = min(row0 + col, q_end - 1);
  const int pos_q = pos0 + my_row;

  // ---- LDS-DMA issue of chunk c into slot c % NS (this wave's P pieces) ----
  // The sequence's block ids are staged in LDS once: a scalar load of a table entry per piece
  // (each followed by its lgkmcnt wait) serialised ~8 round trips into every chunk.
  __shared__ int blk_ids[PREFILL32_MAX_BLOCKS];
  for (int i = threadIdx.x; i < 4 * nchunk; i += 64 * NW) blk_ids[i] = table[min(i, nblk - 1)];
  const unsigned char* kc = reinterpret_cast<const unsigned char*>(g.k);
  const unsigned char* vc = reinterpret_cast<const unsigned char*>(g.v);
  const size_t head_base = static_cast<size_t>(g.layer) * g.num_blocks;
  // lane parts of the source offsets (K piece rows 4 (i & 3) + lane / 16 of a block, its 16-B
  // chunk (lane & 15) ^ row; V^T piece rows d = 32 (i & 3) + lane / 2, half (lane & 1) ^ bit 3 of d)
  const int lane_kx = (lane & 15) ^ (lane >> 4), lane_k = (lane >> 4) * 256;
  const int lane_v = (lane >> 1) * 32 + (((lane ^ (lane >> 4)) & 1) << 4);
  auto issue = [&](int c) __attribute__((always_inline)) {
    unsigned char* slot = ring + (c % NS) * SLOT;
    int blk[P];
#pragma unroll
    for (int pi = 0; pi < P; ++pi) blk[pi] = blk_ids[4 * c + (((w * P + pi) & 15) >> 2)];
#pragma unroll
    for (int pi = 0; pi < P; ++pi) {
      const int i = w * P + pi;  // piece 0..31, wave-uniform
      const int r4 = i & 3;
      const size_t base = ((head_base + __builtin_amdgcn_readfirstlane(blk[pi])) * g.n_kv + kvh) * (BS * HD * 2);
      // K rows 4i .. 4i+3 of the chunk, or V^T rows 32 (i & 3) .. + 31 of block (i & 15) / 4.
      // The DMA as inline asm (M0 = the piece's LDS address): hipcc tracks the builtin's LDS write
      // and put a vmcnt(0) before the next ds_read of the ring -- every chunk then waited for its
      // successor's pieces to land (+4-6 % without).  The ring's own counted wait + barrier in
      // sync() orders the reads.
      const unsigned char* src = i < 16 ? kc + base + (r4 * 1024 + lane_k + ((lane_kx ^ (4 * r4)) << 4))
                                        : vc + base + (r4 * 1024 + lane_v);
      const uint32_t m0v = __builtin_amdgcn_readfirstlane(
          static_cast<uint32_t>(reinterpret_cast<uintptr_t>(slot + (i < 16 ? i * 1024 : KBYTES + (i - 16) * 1024))));
      asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" : : "v"(src), "s"(m0v) : "memory", "m0");
    }
  };

  // Q^T operands: lane (col, h) holds dims 16 kk + 8 h .. + 7 of its row
  bf16x8 bq[HD / 16];
  {
    const bf16_t* qrow = q + (static_cast<size_t>(my_row) * n_q + qh) * HD + 8 * h;
    u32x4 raw[HD / 16];
#pragma unroll
    for (int kk = 0; kk < HD / 16; ++kk) raw[kk] = *reinterpret_cast<const u32x4*>(qrow + 16 * kk);
    // resolve the Q loads before the first DMA: inside the loop the compiler's wait for them
    // would be a vmcnt(0) that drains the ring
#pragma unroll
    for (int kk = 0; kk < HD / 16; ++kk) {
      asm volatile("" : "+v"(raw[kk]));
      bq[kk] = __builtin_bit_cast(bf16x8, raw[kk]);
    }
  }
  __syncthreads();  // block ids staged
#pragma unroll
  for (int c = 0; c < NS - 1; ++c)
    if (c < nchunk) issue(c);

  // K operand addresses: S^T row m = col holds token t0(m) (tile u = 0; u = 1 is t0 + 32, the same
  // swizzle); 16-B chunk 2 kk + h of that row sits at slot (2 kk + h) ^ (t0 & 15), i.e. at byte
  // offset k_lane ^ (kk << 5) (2 kk and h are disjoint bits)
  const int t0 = 16 * (col >> 4) + 8 * ((col >> 2) & 1) + 4 * ((col >> 3) & 1) + (col & 3);
  const int k_lane = t0 * 256 + (((t0 & 15) ^ h) << 4);
  const int v_lane = KBYTES + col * 32 + (((h ^ (col >> 3)) & 1) << 4);

  f32x16 o[HD / 32];
#pragma unroll
  for (int dt = 0; dt < HD / 32; ++dt) o[dt] = f32x16{};
  float m = -INFINITY, lsum = 0.f;  // running max (log2 units, column-uniform), this lane's partial sum

  // chunk c's pieces landed and its successor's slot is free: wait + barrier, then the DMA of
  // chunk c + NS - 1 (every wave runs this for every chunk of the workgroup)
  auto sync = [&](int c) __attribute__((always_inline)) {
    const int ahead = min(NS - 2, nchunk - 1 - c);  // later chunks whose pieces may still fly
    if (ahead >= 2) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * P) : "memory");
    } else if (ahead == 1) {
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();  // ... and every wave is past chunk c - 1: its slot is free
    asm volatile("" ::: "memory");
    if (c + NS - 1 < nchunk) issue(c + NS - 1);
  };
  auto slot_of = [&](int c) { return static_cast<const unsigned char*>(ring + (c % NS) * SLOT); };
  int c = 0;
  float t[32];
  // chunks every row of the wave sees in full, then the diagonal (and context-end) chunks --
  // causal mask, V past the context zeroed -- in loops of their own (no branch on O inside)
  for (; c < n_full; ++c) {
    sync(c);
    attn32_scores<false>(slot_of(c), k_lane, bq, scale_log2, 0, m, lsum, o, t);
    attn32_pv<false>(slot_of(c), v_lane, 0, t, lsum, o);
  }
  for (; c < w_chunks; ++c) {
    sync(c);
    attn32_scores<true>(slot_of(c), k_lane, bq, scale_log2, c * KC + 8 * h - pos_q, m, lsum, o, t);
    attn32_pv<true>(slot_of(c), v_lane, c * KC + 8 * h - ctx, t, lsum, o);
  }
  for (; c < nchunk; ++c) sync(c);  // chunks in the causal future of every row of this wave
  if (!active || row0 + col >= q_end) return;
  {
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(lsum), __float_as_uint(lsum), false, false);
    lsum = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
  }
  const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
  bf16_t* orow = out + (static_cast<size_t>(row0 + col) * n_q + qh) * HD + 4 * h;
#pragma unroll
  for (int dt = 0; dt < HD / 32; ++dt)
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {  // O^T rows d = 32 dt + 8 gq + 4 h + (0..3) of this lane's column
      typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
      bf16x4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = static_cast<__bf16>(o[dt][4 * gq + i] * inv);  // v_cvt_pk_bf16_f32 (RNE)
      *reinterpret_cast<bf16x4*>(orow + 32 * dt + 8 * gq) = v;
    }
}

}  // namespace

// Split size for a decode batch.  Measured on MI355X (tools/bench_ops.py, Qwen3-14B
// geometry, ctx 1700): two 32-token chunks per wave with BOTH chunks' loads issued
// before the first MFMA (256-token items) stream 5.2-5.4 TB/s at B = 160-608, against
// 4.4-4.7 for one chunk per wave (128-token items) -- and halve the split partials the
// merge kernel reads.  (Looping a wave over chunks one at a time was slower: 2-2.6 TB/s.)
constexpr int DEC_CPW = 2;
BCG_API int bcg_decode_split_tokens(int B, int n_kv, int max_tokens) { return DEC_WAVES * CHUNK * DEC_CPW; }
// Partial slots per (row, head): a row's own splits + up to DEC_MAX_SHARED_SPLITS of the
// shared-prefix pass (engine/cascade.py keeps shared tokens / its split within it).
// Only calls with the cascade tables reserve the shared slots (cascade = 0: a plain decode keeps
// the combine kernel's 64-split limit for its own splits, i.e. 16384 tokens of context).
constexpr int DEC_MAX_SHARED_SPLITS = 16;
BCG_API int bcg_decode_max_splits(int max_tokens, int cascade) {
  const int split = DEC_WAVES * CHUNK * DEC_CPW;
  return (max_tokens + split - 1) / split + (cascade ? DEC_MAX_SHARED_SPLITS : 0);
}
// Longest context a decode call supports (the combine kernel reads at most 64 splits per row).
BCG_API int bcg_decode_max_context(int cascade) {
  return (64 - (cascade ? DEC_MAX_SHARED_SPLITS : 0)) * DEC_WAVES * CHUNK * DEC_CPW;
}

// kv_fp8: the caches hold OCP e4m3fn bytes (scale 1) instead of bf16.
BCG_API int bcg_paged_attention_decode(const void* q, const void* k_cache, const void* v_cache, int layer,
                                       int num_blocks, int n_kv, const int* block_tables, int max_blocks,
                                       const int* seq_lens, int B, int n_q, int hd, int block_size,
                                       float scale, float* workspace, int max_splits, int split_tokens,
                                       void* out, int kv_fp8, const int* kv_begin, const int* split_base,
                                       const int* grp_rows, int grp_cap, const int* grp_desc, int max_groups,
                                       const int* items, const int* n_items, int max_items,
                                       int shared_split_tokens, hipStream_t stream) {
  if (block_size != BS || n_q % n_kv || n_q / n_kv > 16 || B <= 0 || B > DEC_MAX_B) return -2;
  // with the cascade a row's own splits start after its shared tokens, in the slots after the
  // shared splits: the host sizes max_splits for both (bcg_decode_max_splits)
  const int own_slots = max_splits - (kv_begin ? DEC_MAX_SHARED_SPLITS : 0);
  if (split_tokens != DEC_WAVES * CHUNK * DEC_CPW || own_slots * split_tokens < max_blocks * BS) return -3;
  if (max_splits > 64) return -3;  // decode_combine_kernel: one lane per split
  Cascade cas{kv_begin, split_base, grp_rows, grp_cap, grp_desc, max_groups, items, n_items, max_items,
              shared_split_tokens};
  if (kv_begin && (!split_base || !grp_rows || !grp_desc || !items || !n_items || grp_cap < 0 || max_groups < 0 ||
                   max_items < 0 || shared_split_tokens <= 0 || shared_split_tokens % CHUNK))
    return -4;
  if (!kv_begin) cas = Cascade{nullptr, nullptr, nullptr, 0, nullptr, 0, nullptr, nullptr, 0, CHUNK};
  KVGeom g{static_cast<const bf16_t*>(k_cache), static_cast<const bf16_t*>(v_cache), layer, num_blocks, n_kv};
  const bf16_t* qb = static_cast<const bf16_t*>(q);
  bf16_t* ob = static_cast<bf16_t*>(out);
  const float sl = scale * LOG2E;
  if (hd == 128 && kv_fp8) {
    launch_decode<128, true, DEC_CPW>(qb, g, block_tables, max_blocks, seq_lens, B, n_q, sl, workspace,
                                             max_splits, ob, cas, stream);
  } else if (hd == 128) {
    launch_decode<128, false, DEC_CPW>(qb, g, block_tables, max_blocks, seq_lens, B, n_q, sl, workspace,
                                              max_splits, ob, cas, stream);
  } else if (hd == 64 && kv_fp8) {
    launch_decode<64, true, DEC_CPW>(qb, g, block_tables, max_blocks, seq_lens, B, n_q, sl, workspace,
                                            max_splits, ob, cas, stream);
  } else if (hd == 64) {
    launch_decode<64, false, DEC_CPW>(qb, g, block_tables, max_blocks, seq_lens, B, n_q, sl, workspace,
                                             max_splits, ob, cas, stream);
  } else {
    return -2;
  }
  return BCG_CHECK_LAUNCH();
}

// nt: 16-row query tiles per wave; only 4 is built (0 = default).
BCG_API int bcg_paged_attention_prefill(const void* q, const void* k_cache, const void* v_cache, int layer,
                                        int num_blocks, int n_kv, const int* block_tables, int max_blocks,
                                        const int* q_start, const int* seq_lens, const int* tiles, int n_tiles,
                                        int n_q, int hd, int block_size, float scale, void* out, int nt,
                                        int kv_fp8, hipStream_t stream) {
  if (block_size != BS || n_q % n_kv || n_tiles <= 0) return -2;
  KVGeom g{static_cast<const bf16_t*>(k_cache), static_cast<const bf16_t*>(v_cache), layer, num_blocks, n_kv};
  const float sl = scale * LOG2E;
  const bf16_t* qb = static_cast<const bf16_t*>(q);
  bf16_t* ob = static_cast<bf16_t*>(out);
  if (nt != 0 && nt != 4) return -2;
  if (hd == 128)
    kv_fp8 ? launch_prefill<128, true>(n_tiles, n_q, qb, g, block_tables, max_blocks, q_start, seq_lens, tiles, sl,
                                       ob, stream)
           : launch_prefill<128, false>(n_tiles, n_q, qb, g, block_tables, max_blocks, q_start, seq_lens, tiles, sl,
                                        ob, stream);
  else if (hd == 64)
    kv_fp8 ? launch_prefill<64, true>(n_tiles, n_q, qb, g, block_tables, max_blocks, q_start, seq_lens, tiles, sl,
                                      ob, stream)
           : launch_prefill<64, false>(n_tiles, n_q, qb, g, block_tables, max_blocks, q_start, seq_lens, tiles, sl,
                                       ob, stream);
  else
    return -2;
  return BCG_CHECK_LAUNCH();
}

// The 32x32 LDS-staged form (prefill_attn32_kernel): `tiles` holds tiles of at most tile_rows
// rows -- 128 (4 waves, 2-slot ring, two workgroups per CU) or 256 (8 waves, 3-slot ring).
// bf16 KV cache and head dim 128 only (-2 otherwise: the caller uses the 16x16 kernel).
constexpr int PREFILL32_NS4 = 2, PREFILL32_NS8 = 3;  // ring slots at 4 / 8 waves (LDS: 2 or 1 workgroups per CU)
BCG_API int bcg_paged_attention_prefill32(const void* q, const void* k_cache, const void* v_cache, int layer,
                                          int num_blocks, int n_kv, const int* block_tables, int max_blocks,
                                          const int* q_start, const int* seq_lens, const int* tiles, int n_tiles,
                                          int n_q, int hd, int block_size, float scale, void* out, int tile_rows,
                                          int kv_fp8, hipStream_t stream) {
  if (block_size != BS || n_kv <= 0 || n_q % n_kv || n_tiles <= 0 || n_q > 65535 || hd != 128 || kv_fp8 ||
      max_blocks > PREFILL32_MAX_BLOCKS || static_cast<long long>(n_tiles) * n_q > 0x7fffffffLL)
    return -2;
  KVGeom g{static_cast<const bf16_t*>(k_cache), static_cast<const bf16_t*>(v_cache), layer, num_blocks, n_kv};
  const float sl = scale * LOG2E;
  const bf16_t* qb = static_cast<const bf16_t*>(q);
  bf16_t* ob = static_cast<bf16_t*>(out);
  const dim3 grid(n_tiles * n_q);  // XCD-grouped 1-D order (see the kernel)
  if (tile_rows == 128)
    hipLaunchKernelGGL((prefill_attn32_kernel<4, PREFILL32_NS4>), grid, dim3(256), 0, stream, qb, g, block_tables,
                       max_blocks, q_start, seq_lens, tiles, n_q, sl, ob, n_tiles);
  else if (tile_rows == 256)
    hipLaunchKernelGGL((prefill_attn32_kernel<8, PREFILL32_NS8>), grid, dim3(512), 0, stream, qb, g, block_tables,
                       max_blocks, q_start, seq_lens, tiles, n_q, sl, ob, n_tiles);
  else
    return -2;
  return BCG_CHECK_LAUNCH();
}
