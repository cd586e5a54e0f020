// 256 x 256 x 64 GEMM, one wave per SIMD with a 256 x 64 wave tile -- the weight operand
// register-fed from a pre-shuffled copy, only X through LDS (gfx950).
//
//   C[M, N] = X[M, K] · W[N, K]^T            (bf16 in, fp32 accumulate, bf16 out)
//
// Sibling of gemm_w4.hip for the prefill projections (SURVEY.md §2.3 K-GEMM-QKV/O/GU/D; the
// reference reaches these GEMMs inside vLLM, byzantine_consensus_game/vllm_agent.py:331/:430).
// What it changes: W4 stages BOTH operands in LDS by LDS-DMA, so per K-tile a CU's LDS takes
// 64 KiB of DMA writes and serves 128 KiB of fragment reads while the MFMAs run -- the LDS
// array is busy most of the K-tile, and each DMA piece stalls its wave (PERF.md, "The four-wave
// 256x256 GEMM").  Here the weights are read in a layout shuffled once at load time
// (`bcg_w4r_shuffle`): for each 64-row panel and 32-deep k-block, the four 16 x 32 MFMA A
// fragments lie lane-major in 4 KiB, so a wave's K-tile of W is ONE contiguous 8 KiB that 8
// `buffer_load_dwordx4` bring straight into the fragment registers (full 128-B lines, no LDS,
// no M0).  The four waves split the tile's N (each all 256 rows x 64 columns), so every W byte
// is loaded once per CU and only X goes through the LDS (a ring of three 32-KiB slots): per
// K-tile and wave 8 LDS-DMA pieces + 8 register loads instead of W4's 16 pieces, half the DMA
// bytes written into the LDS, the same 32 fragment reads.  (A 2 x 2 wave grid with register-fed
// W loads every W panel twice: measured 6-17 % slower than W4, profiles/r6_w4r.)
//
// Schedule (one K-tile t, stream-global index; x slot of tile t = t % 3; every index static,
// the loop body covers two K-tiles so the W register buffer of a tile is static):
//   phase A(t): 64 MFMAs k-step 0 (x0, w[t&1][0])
//               || 16 ds_read_b128 x k-step 1 of tile t -> x1
//               || 8 LDS-DMA pieces X(t+2) -> slot (t+2) % 3
//               || 4 W loads (t+1, k-step 0) -> w[(t+1)&1][0]
//               then s_waitcnt vmcnt(12) lgkmcnt(0); s_barrier
//   phase B(t): 64 MFMAs k-step 1 (x1, w[t&1][1])
//               || 16 ds_read_b128 x k-step 0 of tile t+1 -> x0
//               || 4 W loads (t+1, k-step 1) -> w[(t+1)&1][1]
//               then s_waitcnt vmcnt(4)
// RAW: X(t+1) (issued in A(t-1)) and W(t) k-step 1 (B(t-1)) are older than A(t)'s 12 ops: the
//      vmcnt(12) + barrier after A(t) retire them before phase B(t) reads x0 of tile t+1 and
//      runs on w[t&1][1]; W(t+1) k-step 0 (A(t)) is older than B(t)'s 4 loads: vmcnt(4) at the
//      end of B(t) retires it (and X(t+2)) before A(t+1) runs on it.  LDS-DMA bytes can land
//      after their vmcnt: every X read follows a barrier the issuing waves passed after it.
// WAR: slot (t+2) % 3 = (t-1) % 3 was last read in A(t-1) (x k-step 1, lgkmcnt(0) before the
//      barrier after A(t-1)); w[(t+1)&1][s] was last read by phase s of tile t-1.
// Persistent: one workgroup per CU streams its tiles (items) as one run of K-tiles; the next
// item's first K-tiles are in flight while the last one's epilogue runs.
#include <algorithm>
#include <type_traits>

#include "common.h"

#ifndef W4R_GROUP_M
#define W4R_GROUP_M 8  // m-tiles per tile-order group (L2 reuse of both operands)
#endif

namespace {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int XSLOT = BM * 128;  // one K-tile of X: 256 rows of 128 B
constexpr int NSLOT = 3;
constexpr int NBN = 4, NBM = 16;  // 16-row W blocks / X blocks per wave
enum Epilogue { EPI_STORE = 0, EPI_SILU_MUL = 1, EPI_RESIDUAL = 2 };
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float silu(float g) { return g * __builtin_amdgcn_rcpf(1.f + __expf(-g)); }

__device__ __forceinline__ u16x4 pack4(float a, float b, float c, float d) {
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  const bf16x4 v = {static_cast<__bf16>(a), static_cast<__bf16>(b), static_cast<__bf16>(c), static_cast<__bf16>(d)};
  return __builtin_bit_cast(u16x4, v);
}

// buffer descriptor words (base, stride 0, num_records, raw-buffer config), wave-uniform
__device__ __forceinline__ i32x4 make_srd(const void* base, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  i32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane(static_cast<int>(a & 0xffffffffu));
  r[1] = __builtin_amdgcn_readfirstlane(static_cast<int>(a >> 32) & 0xffff);
  r[2] = __builtin_amdgcn_readfirstlane(static_cast<int>(bytes));
  r[3] = 0x00020000;
  return r;
}

template <int EPI>
__global__ __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_w4r_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ Ws, const bf16_t* __restrict__ bias,
    const bf16_t* __restrict__ residual, bf16_t* __restrict__ C, int M, int N, int K, int ldc, int m_tiles,
    int n_tiles) {
  // ONE shared array (cdna_hip_programming.md "Projection GEMM" item 4a)
  __shared__ __attribute__((aligned(1024))) unsigned char smem[NSLOT * XSLOT];
  const int tiles = m_tiles * n_tiles;
  const int G = gridDim.x;
  const int nk = K / BK;
  const int n_items = (tiles - 1 - static_cast<int>(blockIdx.x)) / G + 1;
  const int total = n_items * nk;  // K-tiles of this workgroup's stream

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;

  // item j -> output tile: XCD-aware bijective remap (item i runs on XCD i % 8), grouped m-tiles
  struct Geo {
    int m0, n0;
  };
  auto geo = [&](int j) {
    const int i = blockIdx.x + j * G;
    const int xcd = i & 7, q = tiles >> 3, rem = tiles & 7;
    const int t = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (i >> 3);
    const int grp = t / (W4R_GROUP_M * n_tiles), in_grp = t % (W4R_GROUP_M * n_tiles);
    const int gm = min(m_tiles - grp * W4R_GROUP_M, W4R_GROUP_M);
    Geo g;
    g.m0 = (grp * W4R_GROUP_M + in_grp % gm) * BM;
    g.n0 = (in_grp / gm) * BN;
    return g;
  };

  // ---- X: LDS-DMA pieces.  Piece i (0..7) of wave w fills slot rows 32 i + 8 w + (lane >> 3),
  // physical chunk lane & 7 <- logical chunk (lane & 7) ^ ((4 w + (lane >> 4)) & 7) (row r's
  // chunk c at c ^ ((r >> 1) & 7): conflict-free fragment reads).  Rows past M read zeros.
  const uint32_t row_bytes = static_cast<uint32_t>(K) * 2;
  const int prow = 8 * wave + (lane >> 3);
  const int pch = ((lane & 7) ^ ((4 * wave + (lane >> 4)) & 7)) * 16;
  const uint32_t voffX = static_cast<uint32_t>(prow) * row_bytes + pch;
  const uint32_t strideX = 32u * row_bytes;
  const uint32_t lds_base = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(smem));
  auto x_srd = [&](const Geo& g) {
    return make_srd(X + static_cast<size_t>(g.m0) * K, static_cast<uint32_t>(M - g.m0) * row_bytes);
  };
  // ---- W: the shuffled copy, [N/64 panels][K/32 k-blocks][4 n-blocks][64 lanes][16 B].  The
  // wave's panel (n0/64 + wave) for K-tile kt is 8 KiB at kt * 8 KiB: load q = 4 s + i is
  // n-block i of k-step s, at q KiB; lane offset lane * 16.  A panel past N reads zeros.
  const uint32_t panel_bytes = static_cast<uint32_t>(K) * 128;
  auto w_srd = [&](const Geo& g) {
    const int p = (g.n0 >> 6) + wave;
    const bool in = p * 64 < N;
    return make_srd(reinterpret_cast<const unsigned char*>(Ws) + static_cast<size_t>(in ? p : 0) * panel_bytes,
                    in ? panel_bytes : 0u);
  };
  uint32_t vW[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) vW[k] = static_cast<uint32_t>(lane) * 16 + k * 4096;

  // cursors: X of stream tile t + 2 (cx), W of stream tile t + 1 (cw)
  int cx_j = 0, cx_k = 0, cw_j = 0, cw_k = 0;
  i32x4 sXc = x_srd(geo(0)), sWc = w_srd(geo(0));
  i32x4 nullX = sXc, nullW = sWc;  // zero-range descriptors: loads past the stream's last tile
  nullX[2] = 0, nullW[2] = 0;
  auto step_cursor = [&](int& j, int& k, i32x4& srd, bool is_x) {
    if (++k == nk) {
      k = 0;
      if (++j < n_items) srd = is_x ? x_srd(geo(j)) : w_srd(geo(j));
    }
  };

  auto piece = [&](int slot, int i, int kt, const i32x4& s) {
    const uint32_t m0v = __builtin_amdgcn_readfirstlane(lds_base + slot * XSLOT + i * 4096 + wave * 1024);
    const uint32_t soff = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(kt) * (BK * 2));
    asm volatile("s_mov_b32 m0, %3\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds"
                 :
                 : "v"(voffX + i * strideX), "s"(s), "s"(soff), "s"(m0v)
                 : "memory", "m0");
  };
  auto wload = [&](bf16x8& dst, int q, int kt, const i32x4& s) {
    const uint32_t soff = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(kt) * 8192);
    switch (q & 3) {  // (immediate offsets: static after unrolling)
      case 0:
        asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(dst) : "v"(vW[q >> 2]), "s"(s), "s"(soff) : "memory");
        break;
      case 1:
        asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen offset:1024"
                     : "=v"(dst) : "v"(vW[q >> 2]), "s"(s), "s"(soff) : "memory");
        break;
      case 2:
        asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen offset:2048"
                     : "=v"(dst) : "v"(vW[q >> 2]), "s"(s), "s"(soff) : "memory");
        break;
      default:
        asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen offset:3072"
                     : "=v"(dst) : "v"(vW[q >> 2]), "s"(s), "s"(soff) : "memory");
        break;
    }
  };

  // x fragment f (16 rows 16 f + fr) of k-step s of the tile in `slot`
  const int rd_sw = (fr >> 1) & 7;
  const int rdA = fr * 128;
  auto read_x = [&](int slot, int s, int f) {
    return *reinterpret_cast<const bf16x8*>(smem + slot * XSLOT + rdA + ((((4 * s + fq) ^ rd_sw)) << 4) + f * 2048);
  };

  // accumulators [n-block][m-block], pinned in AGPRs by the asm MFMA
  f32x4 acc[NBN][NBM];
#pragma unroll
  for (int i = 0; i < NBN; ++i)
#pragma unroll
    for (int j = 0; j < NBM; ++j) acc[i][j] = 0.f;
  auto mf = [&](int idx, const bf16x8 (&w)[NBN], const bf16x8 (&x)[NBM]) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[idx >> 4][idx & 15]) : "v"(w[idx >> 4]), "v"(x[idx & 15]) : "memory");
  };
  auto read_acc = [&](const f32x4& a) {
    f32x4 r;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float v;
      asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(v) : "a"(a[e]));
      r[e] = v;
    }
    return r;
  };
  auto zero_acc = [&]() {
    bf16x8 z = {};
    asm volatile("s_nop 4" : "+v"(z));
#pragma unroll
    for (int i = 0; i < NBN; ++i)
#pragma unroll
      for (int j = 0; j < NBM; ++j)
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %1, 0" : "=a"(acc[i][j]) : "v"(z) : "memory");
  };

  // ---- epilogue (the 16x16 layout of gemm_w4.hip: buffer-addressed, permlane16-swapped 16-B
  // stores / residual loads; SILU: 16-row blocks alternate gate / up of the same 16 features)
  auto epilogue = [&](const Geo& gc) __attribute__((always_inline)) {
    int ln = lane;
    asm volatile("" : "+v"(ln));  // per-lane address math stays out of the K-loop
    const int efr = ln & 15, efq = ln >> 4;
    const int m0 = gc.m0, n0 = gc.n0;
    constexpr bool SILU = EPI == EPI_SILU_MUL;
    constexpr int NP = SILU ? NBN / 4 : NBN / 2;  // 8-column groups per m-block per lane
    const uint32_t ldb = static_cast<uint32_t>(ldc) * 2;
    const int c0 = SILU ? (n0 >> 1) : n0;
    const uint32_t range = static_cast<uint32_t>(M - m0) * ldb;
    const auto rc = __builtin_amdgcn_make_buffer_rsrc(C + static_cast<size_t>(m0) * ldc + c0, 0, range, 0x00020000);
    const uint32_t rowv = static_cast<uint32_t>(efr) * ldb;
    uint32_t colv[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      const int cl = (SILU ? wave * 32 : wave * 64) + (2 * p + (efq & 1)) * 16 + (efq >> 1) * 8;
      colv[p] = SILU || n0 + cl < N ? static_cast<uint32_t>(cl) * 2 : 0x80000000u;
    }
    auto swap8 = [](const float (&a)[4], const float (&b)[4], float (&o)[8]) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a[e]), __float_as_uint(b[e]), false, false);
        o[e] = __uint_as_float(r[0]);
        o[4 + e] = __uint_as_float(r[1]);
      }
    };
    auto pack8 = [](const float (&o)[8]) {
      const u32x2 lo = __builtin_bit_cast(u32x2, pack4(o[0], o[1], o[2], o[3]));
      const u32x2 hi = __builtin_bit_cast(u32x2, pack4(o[4], o[5], o[6], o[7]));
      return u32x4{lo[0], lo[1], hi[0], hi[1]};
    };
    auto store8 = [&](int j, int p, const float (&o)[8]) {
      __builtin_amdgcn_raw_buffer_store_b128(pack8(o), rc, rowv + colv[p] + static_cast<uint32_t>(j * 16) * ldb, 0, 0);
    };
    if constexpr (SILU) {
#pragma unroll
      for (int j = 0; j < NBM; ++j) {
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          float h[2][4];
#pragma unroll
          for (int k = 0; k < 2; ++k) {
            const f32x4 g = read_acc(acc[4 * p + 2 * k][j]), u = read_acc(acc[4 * p + 2 * k + 1][j]);
#pragma unroll
            for (int e = 0; e < 4; ++e) h[k][e] = silu(g[e]) * u[e];
          }
          float o[8];
          swap8(h[0], h[1], o);
          store8(j, p, o);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
      const auto rr_rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<bf16_t*>(EPI == EPI_RESIDUAL ? residual + static_cast<size_t>(m0) * ldc + n0 : C), 0,
          EPI == EPI_RESIDUAL ? range : 0u, 0x00020000);
      u32x4 rq[2][NP];  // the residual groups of m-block j (8 bf16 per lane), next block's ahead
      auto load_rq = [&](int bf, int j) {
        if constexpr (EPI == EPI_RESIDUAL) {
#pragma unroll
          for (int p = 0; p < NP; ++p)
            rq[bf][p] = __builtin_amdgcn_raw_buffer_load_b128(rr_rs, rowv + colv[p] + static_cast<uint32_t>(j * 16) * ldb, 0, 0);
        }
      };
      auto body = [&](auto has_bias) {
        constexpr bool HB = decltype(has_bias)::value;
        u32x4 bq[HB ? NP : 1];
        if constexpr (HB) {
          const auto rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(bias + n0), 0,
                                                            static_cast<uint32_t>(N - n0) * 2, 0x00020000);
#pragma unroll
          for (int p = 0; p < NP; ++p) bq[p] = __builtin_amdgcn_raw_buffer_load_b128(rb, colv[p], 0, 0);
        }
        load_rq(0, 0);
#pragma unroll
        for (int j = 0; j < NBM; ++j) {
          const int bf = j & 1;
          if (j + 1 < NBM) load_rq(bf ^ 1, j + 1);
#pragma unroll
          for (int p = 0; p < NP; ++p) {
            const f32x4 a = read_acc(acc[2 * p][j]), b = read_acc(acc[2 * p + 1][j]);
            const float fa[4] = {a[0], a[1], a[2], a[3]}, fb[4] = {b[0], b[1], b[2], b[3]};
            float o[8];
            swap8(fa, fb, o);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              if constexpr (HB) {
                const uint32_t w = bq[p][e >> 1];
                o[e] += __uint_as_float((e & 1) ? (w & 0xffff0000u) : (w << 16));
              }
              if constexpr (EPI == EPI_RESIDUAL) {
                const uint32_t w = rq[bf][p][e >> 1];
                o[e] += __uint_as_float((e & 1) ? (w & 0xffff0000u) : (w << 16));
              }
            }
            store8(j, p, o);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
      };
      if (bias != nullptr)
        body(std::true_type{});
      else
        body(std::false_type{});
    }
  };

  bf16x8 x0[NBM], x1[NBM];
  bf16x8 w[2][2][NBN];  // [tile parity][k-step][n-block]

  // ---- prologue: X(0), X(1) and W(0) in flight; X(0) landed; x0 of tile 0 read
#pragma unroll
  for (int i = 0; i < 8; ++i) piece(0, i, 0, sXc);
#pragma unroll
  for (int q = 0; q < 8; ++q) wload(w[0][q >> 2][q & 3], q, 0, sWc);
  step_cursor(cx_j, cx_k, sXc, true);  // X cursor -> stream tile 1
  {
    const i32x4 s1 = cx_j < n_items ? sXc : nullX;
#pragma unroll
    for (int i = 0; i < 8; ++i) piece(1, i, cx_k, s1);
  }
  step_cursor(cx_j, cx_k, sXc, true);  // -> stream tile 2
  step_cursor(cw_j, cw_k, sWc, false);  // W cursor -> stream tile 1
  asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");  // X(0) and W(0) landed, X(1) may fly
#pragma unroll
  for (int f = 0; f < NBM; ++f) x0[f] = read_x(0, 0, f);

  Geo gc = geo(0);  // the item whose accumulators are live
  int ktc = 0, jc = 0;

  // one K-tile; P = t & 1 (static), slot = t % 3
  auto ktile = [&](int t, auto parity) __attribute__((always_inline)) {
    constexpr int P = decltype(parity)::value;
    const int slot = t % NSLOT, slot1 = (t + 1) % NSLOT, slot2 = (t + 2) % NSLOT;
    i32x4 sx, sw;
    const bool mx = cx_j < n_items, mw = cw_j < n_items;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      sx[e] = __builtin_amdgcn_readfirstlane(mx ? sXc[e] : nullX[e]),
      sw[e] = __builtin_amdgcn_readfirstlane(mw ? sWc[e] : nullW[e]);
    const int kx = cx_k, kw = cw_k;
    // phase A: k-step 0
#pragma clang loop unroll(full)
    for (int idx = 0; idx < 64; ++idx) {
      mf(idx, w[P][0], x0);
      if (idx < 32 && (idx & 1) == 0) x1[idx >> 1] = read_x(slot, 1, idx >> 1);
      if (idx >= 33 && (idx - 33) % 4 == 0) piece(slot2, (idx - 33) / 4, kx, sx);
      if (idx >= 35 && (idx - 35) % 8 == 0) wload(w[P ^ 1][0][(idx - 35) / 8], (idx - 35) / 8, kw, sw);
    }
    asm volatile("s_waitcnt vmcnt(12) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // phase B: k-step 1
#pragma clang loop unroll(full)
    for (int idx = 0; idx < 64; ++idx) {
      mf(idx, w[P][1], x1);
      if (idx >= 2 && idx < 34 && (idx & 1) == 0) x0[(idx - 2) >> 1] = read_x(slot1, 0, (idx - 2) >> 1);
      if (idx >= 35 && (idx - 35) % 8 == 0) wload(w[P ^ 1][1][(idx - 35) / 8], 4 + (idx - 35) / 8, kw, sw);
    }
    // W(t+1) k-step 0 landed before A(t+1); the MFMA D -> read wait states at the end of the
    // K-tile (the epilogue's accumulator reads come after them)
    asm volatile("s_waitcnt vmcnt(4)\n\ts_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
    step_cursor(cx_j, cx_k, sXc, true);
    step_cursor(cw_j, cw_k, sWc, false);
    if (++ktc == nk) {
      epilogue(gc);
      // none of the epilogue's loads left pending across the back edge (hipcc would drain
      // everything at the next K-tile's top); the next item's loads have had it to land
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
      zero_acc();
      ktc = 0;
      if (++jc < n_items) gc = geo(jc);
    }
  };
  for (int t = 0; t < total; t += 2) {
    ktile(t, std::integral_constant<int, 0>{});
    if (t + 1 < total) ktile(t + 1, std::integral_constant<int, 1>{});
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

int w4r_cus() {
  static int cus[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cus[dev] && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus[dev] = 256;
  return cus[dev] > 0 ? cus[dev] : 256;
}

// [N/64][K/32][4][64][8] <- W[N][K]: lane l of block (panel p, k-block kb, n-block i) holds
// W[64 p + 16 i + (l & 15)][32 kb + 8 (l >> 4) .. +7] (the MFMA A fragment, 16 B).  For the
// SILU form the source rows are gate / up interleaved by 16 (row 32 j + r: gate 16 j + r for
// r < 16, up 16 j + r - 16): `inter` > 0 reads them from W = [gate (inter rows); up].
__global__ void w4r_shuffle_kernel(const bf16_t* __restrict__ W, bf16_t* __restrict__ out, int N, int K, int inter) {
  const int lanes = N / 16 * (K / 32) * 64;  // one 16-B fragment per thread
  for (int g = blockIdx.x * blockDim.x + threadIdx.x; g < lanes; g += gridDim.x * blockDim.x) {
    const int l = g & 63, blk = g >> 6;  // blk = (p * (K/32) + kb) * 4 + i
    const int i = blk & 3, pk = blk >> 2, kb = pk % (K / 32), p = pk / (K / 32);
    int row = 64 * p + 16 * i + (l & 15);
    if (inter > 0) row = (row >> 5) * 16 + (row & 15) + ((row >> 4) & 1) * inter;
    const u16x8 v = *reinterpret_cast<const u16x8*>(W + static_cast<size_t>(row) * K + 32 * kb + 8 * (l >> 4));
    *reinterpret_cast<u16x8*>(out + static_cast<size_t>(g) * 8) = v;
  }
}

template <int EPI>
int launch_w4r(const bf16_t* x, const bf16_t* ws, const bf16_t* bias, const bf16_t* res, bf16_t* c, int M, int N,
               int K, int inter, hipStream_t stream) {
  const int m_tiles = (M + BM - 1) / BM, n_tiles = (N + BN - 1) / BN;
  const int grid = std::min(m_tiles * n_tiles, w4r_cus());
  hipLaunchKernelGGL((gemm_w4r_kernel<EPI>), dim3(grid), dim3(256), 0, stream, x, ws, bias, res, c, M, N, K,
                     EPI == EPI_SILU_MUL ? inter : N, m_tiles, n_tiles);
  return BCG_CHECK_LAUNCH();
}

}  // namespace

// The weight copy bcg_gemm_w4r reads: `out` = N * K bf16.  N % 64 == 0, K % 64 == 0;
// inter > 0 (SILU form): W = [gate; up] with N == 2 * inter, inter % 16 == 0.
BCG_API int bcg_w4r_shuffle(const void* w, void* out, int N, int K, int inter, hipStream_t stream) {
  if (N <= 0 || K <= 0 || N % 64 || K % 64 || (inter > 0 && (N != 2 * inter || inter % 16))) return -2;
  if (1ll * N * K / 8 >= (1ll << 31)) return -2;  // one thread per 16-B fragment (int index)
  const int threads = N / 16 * (K / 32) * 64;
  hipLaunchKernelGGL(w4r_shuffle_kernel, dim3(std::min((threads + 255) / 256, 65536)), dim3(256), 0, stream,
                     static_cast<const bf16_t*>(w), static_cast<bf16_t*>(out), N, K, inter);
  return BCG_CHECK_LAUNCH();
}

// C = X . W^T with the shuffled weights `ws` (bcg_w4r_shuffle); epi 0 = store (+bias),
// 1 = silu(gate) * up into [M, inter] (ws from the SILU form, N == 2 inter, inter % 128 == 0),
// 2 = residual + result (+bias).  N % 64 == 0, K % 64 == 0; one workgroup per CU streams the
// output tiles (the prefill form: no split-K).
BCG_API int bcg_gemm_w4r(int epi, const void* x, const void* ws, const void* bias, const void* residual, void* c,
                         int M, int N, int K, int inter, hipStream_t stream) {
  if (M <= 0 || N <= 0 || K <= 0 || N % 64 || K % BK) return -2;
  // 32-bit buffer offsets: X rows up to a tile past the end, a W panel, the output (+ a masked
  // column's 0x80000000 bias)
  if (2ull * (M + BM) * K >= (1ull << 31) || 128ull * K >= (1ull << 31)) return -2;
  if (2ull * (M + BM) * (epi == EPI_SILU_MUL ? inter : N) >= (1ull << 31)) return -2;
  const bf16_t* xb = static_cast<const bf16_t*>(x);
  const bf16_t* wb = static_cast<const bf16_t*>(ws);
  bf16_t* cb = static_cast<bf16_t*>(c);
  switch (epi) {
    case EPI_STORE:
      return launch_w4r<EPI_STORE>(xb, wb, static_cast<const bf16_t*>(bias), nullptr, cb, M, N, K, inter, stream);
    case EPI_SILU_MUL:
      if (N != 2 * inter || inter % 128) return -2;
      return launch_w4r<EPI_SILU_MUL>(xb, wb, nullptr, nullptr, cb, M, N, K, inter, stream);
    case EPI_RESIDUAL:
      if (!residual) return -2;
      return launch_w4r<EPI_RESIDUAL>(xb, wb, static_cast<const bf16_t*>(bias), static_cast<const bf16_t*>(residual),
                                      cb, M, N, K, inter, stream);
    default:
      return -2;
  }
}
