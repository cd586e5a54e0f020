// Decode-projection GEMM on CDNA4 matrix cores, with fused epilogues.
//
//   C[M, N] = X[M, K] · W[N, K]^T            (bf16 in, fp32 accumulate, bf16 out)
//
// Both operands are K-contiguous (torch Linear layout), so every MFMA fragment is
// one 16-byte row chunk.  SURVEY.md §2.3 K-GEMM-QKV/O/GU/D/LMH; the reference
// reaches these GEMMs inside vLLM (bcg/vllm_agent.py:430).
//
// Structure (one workgroup = BM x BN output tile, 4 waves, WM x WN of them):
//   * K walked in 64-deep tiles; each tile of X (BM rows) and W (BN rows) goes
//     global -> LDS with `global_load_lds` (16 B per lane, no VGPR round trip)
//     into a 2-stage ring: the next tile's loads are issued before the current
//     tile's MFMAs (cdna_hip_programming.md §5.5 T3/T4, "minimum 2-phase");
//   * LDS rows are 128 B; the 16-B chunk c of row r lives at chunk
//     c ^ ((r >> 1) & 7): every 16-lane group of the fragment ds_read_b128 then
//     hits 16 distinct slots of the 256-B bank row (conflict-free).  glds writes
//     linearly, so the swizzle is applied to each lane's SOURCE address (rule 21);
//   * v_mfma_f32_16x16x32_bf16 with the operands swapped (W fragment as A,
//     X fragment as B): a lane ends up with 4 CONSECUTIVE output columns of one
//     row, so the epilogue stores 8 B per lane and sees gate/up (or residual)
//     values of the same columns together;
//   * XCD-aware tile order: the workgroups that share a W tile (same n-tile,
//     all m-tiles) run on one XCD back to back, so each weight byte comes from
//     HBM once and the other m-tiles read it from that XCD's L2.
//
// Epilogues (fused, no extra pass over C):
//   EPI_STORE     C = acc (+ bias)
//   EPI_SILU_MUL  gate_up projection: W rows are [gate (I) ; up (I)], the tile
//                 interleaves 16-row gate/up blocks of the same features, and
//                 the kernel writes h[M, I] = silu(gate) * up directly (K-ACT fused)
//   EPI_RESIDUAL  C = residual + acc (o_proj / down_proj: the residual stream
//                 update of the following add+RMSNorm, fused)
//
// fp8 variant (F8 = true; the fp8-projection path of BASELINE config 5):
//   C[m, n] = xs[m] * ws[n] * sum_k Xq[m, k] Wq[n, k]   (+ bias, + residual)
// with OCP e4m3fn operands, a row-wise activation scale and a per-output-channel weight
// scale (vLLM's dynamic per-token fp8 scheme).  The same 128-B LDS rows then hold 128 K
// elements; each lane's two 16-B fragments of a tile (chunks fq and 4 + fq) form the
// 32-byte operand of ONE block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 (unit E8M0
// scales): 2x the bf16 MFMA rate and half the bytes per K.  A and B use the same
// lane -> k assignment, so the permuted k order inside the instruction cancels.
#include "common.h"

namespace {

constexpr int BK = 64;                 // K elements per tile (128 B per LDS row)

enum Epilogue { EPI_STORE = 0, EPI_SILU_MUL = 1, EPI_RESIDUAL = 2 };

typedef bf16x8 bf16x8s;  // MFMA operand (8 x bf16, 16 B)

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// g * sigmoid(g) with the hardware reciprocal (1 ulp; a true division expands to ~10
// instructions with mode switches per element in the epilogue)
__device__ __forceinline__ float silu(float g) { return g * __builtin_amdgcn_rcpf(1.f + __expf(-g)); }

// Stage `rows` rows x 64 K of a row-major [*, K] bf16 matrix into a linear LDS image
// (row r at byte r*128, swizzled chunks).  Every wave issues rows/32 glds of 8 rows each.
// `src_row(r)` maps a tile row to its global row.
template <int ROWS, int NW, typename RowFn>
__device__ __forceinline__ void stage_tile(unsigned char* lds, const unsigned char* __restrict__ g, int row_bytes,
                                           int k0_bytes, RowFn src_row) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int PER_WAVE = ROWS / (8 * NW);  // 8 rows per glds, NW waves
  static_assert(PER_WAVE >= 1 && ROWS % (8 * NW) == 0, "tile rows per wave");
#pragma unroll
  for (int i = 0; i < PER_WAVE; ++i) {
    const int r = (wave * PER_WAVE + i) * 8 + (lane >> 3);
    const int phys = lane & 7;
    const int c = phys ^ ((r >> 1) & 7);  // logical chunk stored at this slot
    const unsigned char* src = g + static_cast<size_t>(src_row(r)) * row_bytes + k0_bytes + c * 16;
    __builtin_amdgcn_global_load_lds(src, lds + (wave * PER_WAVE + i) * 1024, 16, 0, 0);
  }
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Wait until at most `ahead` tiles' loads (L glds per tile per wave) are outstanding.
template <int L, int MAXAHEAD>
__device__ __forceinline__ void wait_tiles(int ahead) {
  if constexpr (MAXAHEAD <= 0) {
    vm_wait<0>();
  } else {
    if (ahead >= MAXAHEAD) {
      vm_wait<L * MAXAHEAD>();
    } else {
      wait_tiles<L, MAXAHEAD - 1>(ahead);
    }
  }
}

__device__ __forceinline__ void block_sync_lds() {
  // LDS reads retired + every wave here; glds still in flight stay in flight
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));

template <int BM, int BN, int WM, int WN, int S, int EPI, bool F8 = false>
__global__ __launch_bounds__(64 * WM * WN, 1) void gemm_nt_kernel(
    const void* __restrict__ Xv, const void* __restrict__ Wv, const bf16_t* __restrict__ bias,
    const bf16_t* __restrict__ residual, bf16_t* __restrict__ C, float* __restrict__ ws,
    int* __restrict__ counters, int M, int N, int K, int ldc, int inter, int m_tiles, int n_tiles,
    int split_k, const float* __restrict__ x_scale, const float* __restrict__ w_scale) {
  const unsigned char* X = static_cast<const unsigned char*>(Xv);
  const unsigned char* W = static_cast<const unsigned char*>(Wv);
  constexpr int ESZ = F8 ? 1 : 2;      // bytes per element
  constexpr int BKE = 128 / ESZ;       // K elements per tile (one 128-B LDS row)
  constexpr int WTM = BM / WM, WTN = BN / WN;  // wave tile
  constexpr int MT = WTM / 16, NT = WTN / 16;
  constexpr int NW = WM * WN;
  static_assert((NW == 4 || NW == 8) && MT >= 1 && NT >= 1, "4 or 8 waves");
  static_assert(EPI != EPI_SILU_MUL || NT % 2 == 0, "gate/up pairs per wave");
  static_assert(S >= 2, "at least double buffering");
  static_assert(MT + NT <= 15, "lgkmcnt counts at most 15 LDS reads");
  static_assert(!F8 || EPI != EPI_SILU_MUL, "fp8: store / residual epilogues");
  constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128, STAGE = A_BYTES + B_BYTES;
  constexpr int L = BM / (8 * NW) + BN / (8 * NW);  // glds per tile per wave
  // ONE shared array for everything (a second __shared__ object can make hipcc drain
  // vmcnt before every ds_read: cdna_hip_programming.md "Projection GEMM" item 4a)
  __shared__ __attribute__((aligned(1024))) unsigned char smem[S * STAGE];

  // ---- XCD-aware order: bijective remap, then (n-tile, m-tile, k-split) with the
  //      splits of a tile and the m-tiles of an n-tile adjacent on one XCD ----
  const int nwg = m_tiles * n_tiles * split_k;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, rem = nwg & 7;
  const int r_id = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (bid >> 3);
  const int split = r_id % split_k;
  const int tile = r_id / split_k;
  const int m_tile = tile % m_tiles, n_tile = tile / m_tiles;
  const int m0 = m_tile * BM, n0 = n_tile * BN;
  const int nk_all = K / BKE;
  const int kt0 = split * nk_all / split_k, kt1 = (split + 1) * nk_all / split_k;
  const int nk = kt1 - kt0;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int fr = lane & 15, fq = lane >> 4;

  auto x_row = [&](int r) { return min(m0 + r, M - 1); };  // clamped rows are discarded
  auto w_row = [&](int r) {
    if constexpr (EPI == EPI_SILU_MUL) {  // 16-row blocks alternate gate / up of the same features
      const int blk = r >> 4;
      const int feat = (n0 >> 1) + (blk >> 1) * 16 + (r & 15);
      return (blk & 1) ? inter + feat : feat;
    } else {
      return n0 + r;
    }
  };
  auto issue = [&](int t) {  // tile t (relative) -> stage t % S
    unsigned char* st = smem + (t % S) * STAGE;
    const int k0b = (kt0 + t) * 128;
    stage_tile<BM, NW>(st, X, K * ESZ, k0b, x_row);
    stage_tile<BN, NW>(st + A_BYTES, W, K * ESZ, k0b, w_row);
  };

  f32x4 acc[NT][MT];
#pragma unroll
  for (int i = 0; i < NT; ++i)
#pragma unroll
    for (int j = 0; j < MT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragments of one 32-deep k-step: this wave's MT x-rows blocks and NT w-rows blocks
  auto read_frags = [&](int t, int sstep, bf16x8s (&xa)[MT], bf16x8s (&wb)[NT]) {
    const unsigned char* As = smem + (t % S) * STAGE;
    const unsigned char* Bs = As + A_BYTES;
    const int chunk = 4 * sstep + fq;
#pragma unroll
    for (int j = 0; j < MT; ++j) {
      const int r = wm * WTM + j * 16 + fr;
      xa[j] = *reinterpret_cast<const bf16x8s*>(As + r * 128 + swz(r, chunk) * 16);
    }
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      const int r = wn * WTN + i * 16 + fr;
      wb[i] = *reinterpret_cast<const bf16x8s*>(Bs + r * 128 + swz(r, chunk) * 16);
    }
  };
  // fp8: the two k-steps' fragments of a tile are one 32-byte operand (K = 128)
  auto mfmas8 = [&](const bf16x8s (&xa)[MT], const bf16x8s (&wb)[NT], const bf16x8s (&xb)[MT],
                    const bf16x8s (&wc)[NT]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      const i32x4 w0 = __builtin_bit_cast(i32x4, wb[i]), w1 = __builtin_bit_cast(i32x4, wc[i]);
      const i32x8 wop = {w0[0], w0[1], w0[2], w0[3], w1[0], w1[1], w1[2], w1[3]};
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        const i32x4 x0 = __builtin_bit_cast(i32x4, xa[j]), x1 = __builtin_bit_cast(i32x4, xb[j]);
        const i32x8 xop = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
        // formats 0/0 = e4m3 x e4m3; E8M0 scale 127 = 1.0 for both operands
        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wop, xop, acc[i][j], 0, 0, 0, 127, 0, 127);
      }
    }
    __builtin_amdgcn_s_setprio(0);
  };
  auto mfmas = [&](const bf16x8s (&xa)[MT], const bf16x8s (&wb)[NT]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int j = 0; j < MT; ++j)  // D[n][m]: W fragment as A, X fragment as B
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wb[i], xa[j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // Software pipeline: while the MFMAs of one 32-deep k-step run, the LDS reads of the
  // next one (the second half of this tile, or the first half of the next tile) are in
  // flight -- the 8 waves pass the same barriers, so without this every wave would wait
  // out the LDS traffic of all waves before its first MFMA of each step.
  // Tile t lives in stage t % S; S-1 tiles are always in flight ahead of the one read.
#pragma unroll
  for (int t = 0; t < S - 1; ++t)
    if (t < nk) issue(t);
  bf16x8s xa0[MT], wb0[NT], xa1[MT], wb1[NT];
  wait_tiles<L, S - 2>(min(nk, S - 1) - 1);
  block_sync_lds();
  if (S - 1 < nk) issue(S - 1);
  read_frags(0, 0, xa0, wb0);
  for (int kt = 0; kt < nk; ++kt) {
    read_frags(kt, 1, xa1, wb1);
    if constexpr (F8) {  // one K = 128 MFMA per block pair over both k-steps' fragments
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      mfmas8(xa0, wb0, xa1, wb1);
      if (kt + 1 < nk) {
        wait_tiles<L, S - 2>(min(nk, kt + S) - kt - 2);
        block_sync_lds();
        if (kt + S < nk) issue(kt + S);
        read_frags(kt + 1, 0, xa0, wb0);
      }
      continue;
    }
    asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(MT + NT) : "memory");  // k-step 0 landed
    mfmas(xa0, wb0);
    if (kt + 1 < nk) {
      // tile kt+1 landed for every wave, and every wave is done reading tile kt
      wait_tiles<L, S - 2>(min(nk, kt + S) - kt - 2);
      block_sync_lds();  // (its lgkmcnt(0) also retires this wave's k-step-1 reads)
      if (kt + S < nk) issue(kt + S);  // into tile kt's stage
      read_frags(kt + 1, 0, xa0, wb0);
    } else {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    mfmas(xa1, wb1);
  }

  // ---- split-K: partial tiles -> workspace; the last-arriving split reduces ----
  // Hand-off without L2 maintenance (cdna_hip_programming.md §6 Guideline 16, R1):
  // partials are stored WRITE-THROUGH (sc1), every wave drains vmcnt, barrier, one
  // relaxed agent-scope ticket; the reducer reads the other slabs with sc1 loads.  (An
  // agent-scope release/acquire pair is buffer_wbl2 + buffer_inv on gfx950: an L2
  // write-back per episode.)
  if (split_k > 1) {
    typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
    float* slab = ws + static_cast<size_t>(tile) * split_k * (BM * BN);
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(slab, 0, split_k * BM * BN * 4, 0x00020000);
    const int tid = threadIdx.x;
    __syncthreads();  // every wave is past its last ds_read: smem is reusable as the flag slot
    int* flag = reinterpret_cast<int*>(smem);
    // block (i, j) of this wave: 256 floats, lane-major (4 per lane = one 16-B access)
#pragma unroll
    for (int i = 0; i < NT; ++i)
#pragma unroll
      for (int j = 0; j < MT; ++j) {
        const int off = (split * (BM * BN) + ((wave * NT + i) * MT + j) * 256 + lane * 4) * 4;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, acc[i][j]), rs, off, 0, 16 /*sc1*/);
      }
    vm_wait<0>();
    __syncthreads();
    if (tid == 0) {
      const int prev = __hip_atomic_fetch_add(&counters[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = prev == split_k - 1;
      if (last) __hip_atomic_store(&counters[tile], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
      flag[0] = last;
    }
    __syncthreads();
    if (!flag[0]) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below
    for (int sp = 0; sp < split_k; ++sp) {
      if (sp == split) continue;
#pragma unroll
      for (int i = 0; i < NT; ++i)
#pragma unroll
        for (int j = 0; j < MT; ++j) {
          const int off = (sp * (BM * BN) + ((wave * NT + i) * MT + j) * 256 + lane * 4) * 4;
          acc[i][j] += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16 /*sc1*/));
        }
    }
  }

  // ---- epilogue: lane holds D[n = 4fq + e][m = fr] of every (i, j) block, e = 0..3 ----
#pragma unroll
  for (int j = 0; j < MT; ++j) {
    const int m = m0 + wm * WTM + j * 16 + fr;
    if (m >= M) continue;
    if constexpr (EPI == EPI_SILU_MUL) {
#pragma unroll
      for (int i = 0; i < NT; i += 2) {  // (gate, up) block pairs of the same 16 features
        const int tile_row = wn * WTN + i * 16;
        const int feat = (n0 >> 1) + (tile_row >> 5) * 16 + 4 * fq;
        u16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = f2bf(silu(acc[i][j][e]) * acc[i + 1][j][e]);
        *reinterpret_cast<u16x4*>(C + static_cast<size_t>(m) * ldc + feat) = o;
      }
    } else {
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        const int n = n0 + wn * WTN + i * 16 + 4 * fq;
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
        if constexpr (F8) {  // dequantise: row scale x column scales
          const float xs = x_scale[m];
          const f32x4 wsc = *reinterpret_cast<const f32x4*>(w_scale + n);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] *= xs * wsc[e];
        }
        if (bias != nullptr) {
          const u16x4 b = *reinterpret_cast<const u16x4*>(bias + n);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += bf2f(b[e]);
        }
        if constexpr (EPI == EPI_RESIDUAL) {
          const u16x4 rr = *reinterpret_cast<const u16x4*>(residual + static_cast<size_t>(m) * ldc + n);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += bf2f(rr[e]);
        }
        u16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = f2bf(v[e]);
        *reinterpret_cast<u16x4*>(C + static_cast<size_t>(m) * ldc + n) = o;
      }
    }
  }
}

struct TileCfg {
  int bm, bn, stages;
};
// 0 = 128x128, 1 = 64x128, 2 = 128x64, 3 = 256x128, 4 = 64x256, 5 = 64x64, 6 = 32x128 (4 waves);
// 7 = 256x128, 8 = 128x256, 9 = 128x128 (8 waves: two per SIMD, one's MFMAs cover the other's LDS reads)
constexpr TileCfg CFGS[] = {{128, 128, 4}, {64, 128, 5}, {128, 64, 5},  {256, 128, 3}, {64, 256, 4},
                            {64, 64, 6},   {32, 128, 6}, {256, 128, 3}, {128, 256, 3}, {128, 128, 4}};
constexpr int N_CFG = sizeof(CFGS) / sizeof(CFGS[0]);

template <int BM, int BN, int WM, int WN, int S, int EPI, bool F8 = false>
int launch(const void* x, const void* w, const void* bias, const void* res, void* c, float* ws, int* cnt, int M,
           int N, int K, int inter, int split_k, hipStream_t stream, const float* xs = nullptr,
           const float* wsc = nullptr) {
  const int m_tiles = (M + BM - 1) / BM, n_tiles = N / BN;
  const int ldc = EPI == EPI_SILU_MUL ? inter : N;
  hipLaunchKernelGGL((gemm_nt_kernel<BM, BN, WM, WN, S, EPI, F8>), dim3(m_tiles * n_tiles * split_k),
                     dim3(64 * WM * WN), 0, stream, x, w, static_cast<const bf16_t*>(bias),
                     static_cast<const bf16_t*>(res), static_cast<bf16_t*>(c), ws, cnt, M, N, K, ldc, inter, m_tiles,
                     n_tiles, split_k, xs, wsc);
  return BCG_CHECK_LAUNCH();
}

template <int EPI, bool F8 = false>
int dispatch(int cfg, const void* x, const void* w, const void* bias, const void* res, void* c, float* ws, int* cnt,
             int M, int N, int K, int inter, int sk, hipStream_t s, const float* xs = nullptr,
             const float* wsc = nullptr) {
  switch (cfg) {
    case 0: return launch<128, 128, 2, 2, 4, EPI, F8>(x, w, bias, res, c, ws, cnt, M, N, K, inter, sk, s, xs, wsc);
    case 1: return launch<64, 128, 1, 4, 5, EPI, F8>(x, w, bias, res, c, ws, cnt, M, N, K, inter, sk, s, xs, wsc);
    case 2: return launch<128, 64, 2, 2, 5, EPI, F8>(x, w, bias, res, c, ws, cnt, M, N, K, inter, sk, s, xs, wsc);
    case 3: return launch<256, 128, 4, 1, 3, EPI, F8>(x, w, bias, res, c, ws, cnt, M, N, K, inter, sk, s, xs, wsc);
    case 4: return launch<64, 256, 1, 4, 4, EPI, F8>(x, w, bias, res, c, ws, cnt, M, N, K, inter, sk, s, xs, wsc);
    case 5: return launch<64, 64, 2, 2, 6, EPI, F8>(x, w, bias, res, c, ws, cnt, M, N, K, inter, sk, s, xs, wsc);
    case 6: return launch<32, 128, 1, 4, 6, EPI, F8>(x, w, bias, res, c, ws, cnt, M, N, K, inter, sk, s, xs, wsc);
    case 7: return launch<256, 128, 4, 2, 3, EPI, F8>(x, w, bias, res, c, ws, cnt, M, N, K, inter, sk, s, xs, wsc);
    case 8: return launch<128, 256, 2, 4, 3, EPI, F8>(x, w, bias, res, c, ws, cnt, M, N, K, inter, sk, s, xs, wsc);
    case 9: return launch<128, 128, 2, 4, 4, EPI, F8>(x, w, bias, res, c, ws, cnt, M, N, K, inter, sk, s, xs, wsc);
    default: return -2;
  }
}

}  // namespace

BCG_API int bcg_gemm_pp(int epi, const void* x, const void* w, const void* bias, const void* residual, void* c,
                        void* ws, void* counters, int M, int N, int K, int inter, int split_k, hipStream_t stream);
constexpr int PP_CFG = N_CFG;  // the 256 x 256 ping-pong kernel (gemm_pp.hip)
BCG_API int bcg_gemm_w4(int epi, const void* x, const void* w, const void* bias, const void* residual, void* c,
                        void* ws, void* counters, int M, int N, int K, int inter, int split_k, hipStream_t stream);
BCG_API int bcg_gemm_w4_fp8(int epi, const void* xq, const void* wq, const float* x_scale, const float* w_scale,
                            const void* bias, const void* residual, void* c, void* ws, void* counters, int M, int N,
                            int K, int split_k, hipStream_t stream);
constexpr int W4_CFG = N_CFG + 1;  // 256 x 256, four 128 x 128 waves, LDS-DMA fed (gemm_w4.hip)

// Tile configurations: see CFGS (BM x BN, pipeline stages); PP_CFG = gemm_pp.hip.
BCG_API int bcg_gemm_tile(int cfg, int* bm, int* bn) {
  if (cfg == PP_CFG || cfg == W4_CFG) {
    *bm = *bn = 256;
    return 0;
  }
  if (cfg < 0 || cfg >= N_CFG) return -2;
  *bm = CFGS[cfg].bm;
  *bn = CFGS[cfg].bn;
  return 0;
}

BCG_API int bcg_gemm_num_cfgs() { return N_CFG + 2; }

// epi: 0 = store (+bias), 1 = silu(gate)*up into [M, inter], 2 = residual + acc.
// split_k > 1: fp32 partial tiles in `ws` (>= m_tiles*n_tiles*split_k*BM*BN floats) and one
// zero-initialised int counter per output tile in `counters` (left zeroed by every launch).
// Requirements (checked by the caller): K % 64 == 0, K/64 >= split_k; N % BN == 0; EPI 1:
// N == 2*inter and inter % (BN/2) == 0; all pointers 16-B aligned, rows contiguous.
BCG_API int bcg_gemm_nt(int cfg, int epi, const void* x, const void* w, const void* bias, const void* residual,
                        void* c, void* ws, void* counters, int M, int N, int K, int inter, int split_k,
                        hipStream_t stream) {
  if (cfg == PP_CFG) return bcg_gemm_pp(epi, x, w, bias, residual, c, ws, counters, M, N, K, inter, split_k, stream);
  if (cfg == W4_CFG) return bcg_gemm_w4(epi, x, w, bias, residual, c, ws, counters, M, N, K, inter, split_k, stream);
  if (M <= 0 || K % BK || K <= 0 || split_k < 1 || K / BK < split_k) return -2;
  if (split_k > 1 && (!ws || !counters)) return -2;
  int bm, bn;
  if (bcg_gemm_tile(cfg, &bm, &bn)) return -2;
  if (N % bn) return -2;
  float* wsf = static_cast<float*>(ws);
  int* cnt = static_cast<int*>(counters);
  switch (epi) {
    case EPI_STORE: return dispatch<EPI_STORE>(cfg, x, w, bias, residual, c, wsf, cnt, M, N, K, inter, split_k, stream);
    case EPI_SILU_MUL:
      if (N != 2 * inter || inter % (bn / 2)) return -2;
      return dispatch<EPI_SILU_MUL>(cfg, x, w, nullptr, nullptr, c, wsf, cnt, M, N, K, inter, split_k, stream);
    case EPI_RESIDUAL:
      if (!residual) return -2;
      return dispatch<EPI_RESIDUAL>(cfg, x, w, bias, residual, c, wsf, cnt, M, N, K, inter, split_k, stream);
    default: return -2;
  }
}

// fp8 (e4m3fn) projection GEMM: C = x_scale[m] * w_scale[n] * (Xq . Wq^T) (+ bias) (+ residual).
// epi: 0 = store, 2 = residual + result.  Requirements: K % 128 == 0, K/128 >= split_k,
// N % BN == 0 (cfg's tile), x_scale [M] / w_scale [N] fp32, pointers 16-B aligned; split-K
// workspace / counters as bcg_gemm_nt.
BCG_API int bcg_gemm_pp_fp8(int epi, const void* xq, const void* wq, const float* x_scale, const float* w_scale,
                            const void* bias, const void* residual, void* c, void* ws, void* counters, int M, int N,
                            int K, int split_k, hipStream_t stream);

BCG_API int bcg_gemm_nt_fp8(int cfg, int epi, const void* xq, const void* wq, const float* x_scale,
                            const float* w_scale, const void* bias, const void* residual, void* c, void* ws,
                            void* counters, int M, int N, int K, int split_k, hipStream_t stream) {
  if (cfg == PP_CFG)  // the 256 x 256 ping-pong kernel's fp8 form (prefill M)
    return bcg_gemm_pp_fp8(epi, xq, wq, x_scale, w_scale, bias, residual, c, ws, counters, M, N, K, split_k, stream);
  if (cfg == W4_CFG)  // the four-wave 256 x 256 kernel's fp8 form (32x32x64 block-scaled MFMAs)
    return bcg_gemm_w4_fp8(epi, xq, wq, x_scale, w_scale, bias, residual, c, ws, counters, M, N, K, split_k, stream);
  if (M <= 0 || K % 128 || K <= 0 || split_k < 1 || K / 128 < split_k || !x_scale || !w_scale) return -2;
  if (split_k > 1 && (!ws || !counters)) return -2;
  if (cfg < 0 || cfg >= N_CFG || N % CFGS[cfg].bn) return -2;
  float* wsf = static_cast<float*>(ws);
  int* cnt = static_cast<int*>(counters);
  switch (epi) {
    case EPI_STORE:
      return dispatch<EPI_STORE, true>(cfg, xq, wq, bias, residual, c, wsf, cnt, M, N, K, 0, split_k, stream,
                                       x_scale, w_scale);
    case EPI_RESIDUAL:
      if (!residual) return -2;
      return dispatch<EPI_RESIDUAL, true>(cfg, xq, wq, bias, residual, c, wsf, cnt, M, N, K, 0, split_k, stream,
                                          x_scale, w_scale);
    default: return -2;
  }
}
