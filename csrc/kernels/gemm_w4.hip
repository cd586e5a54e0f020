// 256 x 256 x 64 GEMM, ONE wave per SIMD with a 128 x 128 wave tile, LDS-DMA fed (gfx950).
//
//   C[M, N] = X[M, K] · W[N, K]^T            (bf16 in, fp32 accumulate, bf16 out)
//
// The prefill-projection kernel (SURVEY.md §2.3 K-GEMM-QKV/O/GU/D; the reference reaches these
// GEMMs inside vLLM, byzantine_consensus_game/vllm_agent.py:331/:430).  Why this shape:
//   * the 8-wave ping-pong kernel (gemm_pp.hip) gives each wave a 128 x 64 tile, so a CU reads
//     192 KiB of fragments out of LDS per 64-deep K-tile; four waves of 128 x 128 read 128 KiB
//     for the same FLOPs (a wave's LDS bytes scale with rows + columns of its tile);
//   * 128 x 128 needs 256 fp32 accumulators per lane: only one wave per SIMD has the registers
//     (512 = 256 accumulators in AGPRs + two k-steps of fragments + addresses);
//   * the K-tiles come in by LDS-DMA (`buffer_load_dwordx4 ... lds`: no VGPR staging, no
//     ds_write), one SGPR offset per piece, so the only VGPR per piece is a constant per-lane
//     row offset;  the register-staged form of this tile (csrc/experimental/gemm_rs.hip) lost
//     on its 16 ds_write_b128 per K-tile (PERF.md "Round 3: the 256x256 feed");
//   * the disassembly of hipBLASLt's own MT256x256x64 kernel on this image (the library the
//     table used to pick for these shapes) has exactly these resources: 256 threads, 256
//     AGPR accumulators, 16x16x32 MFMAs, LDS-DMA loads -- the schedule below is our own.
//
// Schedule (one K-tile t, stage s = t & 1 of a 2 x 64 KiB LDS ring; every index static):
//   phase A: 64 MFMAs of k-step 0 (fragments x0/w0 in registers)
//            || 16 ds_read_b128 of k-step 1 of tile t (stage s) -> x1/w1
//            then  s_waitcnt vmcnt(0) lgkmcnt(0); s_barrier
//   phase B: 64 MFMAs of k-step 1 (x1/w1)
//            || 16 LDS-DMA pieces of tile t+2 -> stage s
//            || 16 ds_read_b128 of k-step 0 of tile t+1 (stage s^1) -> x0/w0
// RAW: tile t+1's pieces were issued in phase B of tile t-1 and are waited for by every wave
//      before the barrier that precedes their first read (phase B of tile t).
// WAR: stage s was last read by tile t's k-step-0 reads (phase B of t-1) and k-step-1 reads
//      (phase A of t); both drained (lgkmcnt(0)) by every wave before the barrier of tile t,
//      after which tile t+2's pieces are issued.
// One barrier per K-tile, a piece has 1.5 phases (~1500 cycles) to land.
//
// LDS: rows of 128 B (64 bf16 of K), the 16-B chunk c of row r at c ^ ((r >> 1) & 7): the
// fragment ds_read_b128s are conflict-free (gemm.hip); LDS-DMA writes lane-linearly, so the
// swizzle is applied to each lane's SOURCE chunk.  Operands swapped in the MFMA (W fragment
// as A) so a lane holds 4 consecutive output columns of one row.  XCD-aware grouped tile
// order and last-arriver split-K as gemm_pp.hip; the same host contract (bcg_gemm_w4).
#include <type_traits>

#include "common.h"

#ifndef W4_GROUP_M
#define W4_GROUP_M 8  // m-tiles per tile-order group (L2 reuse of both operands)
#endif
// schedule knobs: first MFMA slot and slot stride of each memory-op stream (64 slots/phase)
#ifndef W4_RA0
#define W4_RA0 0  // phase A: k-step-1 reads
#endif
#ifndef W4_RAS
#define W4_RAS 2
#endif
#ifndef W4_DB0
#define W4_DB0 0  // phase B: LDS-DMA pieces
#endif
#ifndef W4_DBS
#define W4_DBS 3
#endif
#ifndef W4_RB0
#define W4_RB0 1  // phase B: k-step-0 reads of the next tile
#endif
#ifndef W4_RBS
#define W4_RBS 3
#endif

namespace {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int A_BYTES = BM * 128, STAGE = A_BYTES + BN * 128;  // 64 KiB
enum Epilogue { EPI_STORE = 0, EPI_SILU_MUL = 1, EPI_RESIDUAL = 2 };
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

static_assert(W4_RA0 + 15 * W4_RAS < 64 && W4_DB0 + 15 * W4_DBS < 64 && W4_RB0 + 15 * W4_RBS < 64,
              "each stream fits its phase");

__device__ __forceinline__ float silu(float g) { return g / (1.f + __expf(-g)); }

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

#ifdef W4_STAMPS
__device__ uint64_t w4_stamps[1 << 16];  // [workgroup][wave][phase A, wait, phase B, K-tiles]
#endif

template <int EPI>
__global__ __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_w4_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ W, const bf16_t* __restrict__ bias,
    const bf16_t* __restrict__ residual, bf16_t* __restrict__ C, float* __restrict__ ws,
    int* __restrict__ counters, int M, int N, int K, int ldc, int inter, int m_tiles, int n_tiles,
    int split_k) {
  // ONE shared array (cdna_hip_programming.md "Projection GEMM" item 4a)
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * STAGE];

  // ---- XCD-aware order (bijective remap), grouped m-tiles, then (tile, k-split) ----
  const int nwg = m_tiles * n_tiles * split_k;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, rem = nwg & 7;
  const int r_id = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (bid >> 3);
  const int split = r_id % split_k;
  const int tile = r_id / split_k;
  const int grp = tile / (W4_GROUP_M * n_tiles), in_grp = tile % (W4_GROUP_M * n_tiles);
  const int gm = min(m_tiles - grp * W4_GROUP_M, W4_GROUP_M);
  const int m_tile = grp * W4_GROUP_M + in_grp % gm, n_tile = in_grp / gm;
  const int m0 = m_tile * BM, n0 = n_tile * BN;
  const int nk_all = K / BK;
  const int kt0 = split * nk_all / split_k;
  const int nk = (split + 1) * nk_all / split_k - kt0;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1;
  const int fr = lane & 15, fq = lane >> 4;

  // ---- LDS-DMA pieces: piece i (0..7) of wave w fills stage rows 32 i + 8 w + (lane >> 3),
  // physical chunk lane & 7 <- logical chunk (lane & 7) ^ ((4 w + (lane >> 4)) & 7).  Rows past
  // M / N fall outside the descriptor's range and read zeros (never stored).
  const uint32_t row_bytes = static_cast<uint32_t>(K) * 2;
  const int prow = 8 * wave + (lane >> 3);
  const int pch = ((lane & 7) ^ ((4 * wave + (lane >> 4)) & 7)) * 16;
  const i32x4 srdX = make_srd(X, static_cast<uint32_t>(M) * row_bytes);
  const i32x4 srdW = make_srd(W, static_cast<uint32_t>(EPI == EPI_SILU_MUL ? 2 * inter : N) * row_bytes);
  const uint32_t voffX = static_cast<uint32_t>(m0 + prow) * row_bytes + pch;
  // SILU: 16-row blocks of the tile alternate gate / up of the same 16 features, so stage row
  // 32 i + r (r < 32) holds W row (r >> 4) * inter + n0/2 + 16 i + (r & 15)
  const uint32_t voffW =
      static_cast<uint32_t>(EPI == EPI_SILU_MUL ? (wave >> 1) * inter + (n0 >> 1) + (prow & 15) : n0 + prow) *
          row_bytes + pch;
  const uint32_t strideX = 32u * row_bytes;
  const uint32_t strideW = (EPI == EPI_SILU_MUL ? 16u : 32u) * row_bytes;
  // the row part of a piece's offset stays in the VGPR offset: only that is range-checked
  // (the SGPR offset carries the K-tile)
  uint32_t vX[8], vW[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) vX[i] = voffX + i * strideX, vW[i] = voffW + i * strideW;
  const uint32_t lds_base = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(smem));
  // piece q (0..15) of tile t into `stage`: q < 8 X piece q, else W piece q - 8
  auto dma = [&](int t, int stage, int q, const i32x4& sX, const i32x4& sW) {
    const uint32_t kb = static_cast<uint32_t>(kt0 + t) * (BK * 2);
    const bool isx = q < 8;
    const int i = q & 7;
    const uint32_t soff = __builtin_amdgcn_readfirstlane(kb);
    const uint32_t m0v = __builtin_amdgcn_readfirstlane(lds_base + stage * STAGE + (isx ? 0 : A_BYTES) +
                                                        i * 4096 + wave * 1024);
    if (isx) {
      asm volatile("s_mov_b32 m0, %3\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds"
                   :
                   : "v"(vX[i]), "s"(sX), "s"(soff), "s"(m0v)
                   : "memory", "m0");
    } else {
      asm volatile("s_mov_b32 m0, %3\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds"
                   :
                   : "v"(vW[i]), "s"(sW), "s"(soff), "s"(m0v)
                   : "memory", "m0");
    }
  };

  // ---- fragments of a 32-deep k-step: x block f = stage row wm*128 + 16 f + fr, w block f =
  // stage row A_BYTES/128 + wn*128 + 16 f + fr; chunk 4 s + fq, swizzled by (fr >> 1) & 7
  const int rd_sw = (fr >> 1) & 7;
  const int rdA = (wm * 128 + fr) * 128, rdB = A_BYTES + (wn * 128 + fr) * 128;
  auto read_frag = [&](int stage, int s, int f, bf16x8 (&xf)[8], bf16x8 (&wf)[8]) {
    const int off = stage * STAGE + (((4 * s + fq) ^ rd_sw) << 4) + (f & 7) * 2048 + (f < 8 ? rdA : rdB);
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(smem + off);
    if (f < 8)
      xf[f] = v;
    else
      wf[f - 8] = v;
  };

  f32x4 acc[8][8];  // [n-block][m-block], pinned in AGPRs by the asm MFMA below
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // "memory" keeps the MFMAs in source order with the LDS reads and DMA issued between them;
  // the builtin form lets hipcc cycle the accumulators through a few AGPRs (gemm_rs.hip)
  auto mf = [&](int idx, const bf16x8 (&xf)[8], const bf16x8 (&wf)[8]) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                 : "+a"(acc[idx >> 3][idx & 7])
                 : "v"(wf[idx >> 3]), "v"(xf[idx & 7])
                 : "memory");
  };

  bf16x8 x0[8], w0[8], x1[8], w1[8];
  // ---- prologue: tiles 0 and 1 in flight, tile 0 landed, k-step 0 of tile 0 in registers ----
#pragma unroll
  for (int q = 0; q < 16; ++q) dma(0, 0, q, srdX, srdW);
  if (nk > 1) {
#pragma unroll
    for (int q = 0; q < 16; ++q) dma(1, 1, q, srdX, srdW);
    asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  }
#pragma unroll
  for (int f = 0; f < 16; ++f) read_frag(0, 0, f, x0, w0);

  // phase B of tile t.  Past the last tile the pieces go through a zero-range descriptor: no
  // memory traffic, the zeros land in a stage nobody reads -- branch-free, one body (a
  // branch around the pieces, or two copies of the phase, made hipcc spill the accumulators)
  i32x4 nullX = srdX, nullW = srdW;
  nullX[2] = 0, nullW[2] = 0;
  auto phase_b = [&](int t, int cur) {
    const bool more = t + 2 < nk;
    i32x4 sX, sW;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      sX[e] = __builtin_amdgcn_readfirstlane(more ? srdX[e] : nullX[e]),
      sW[e] = __builtin_amdgcn_readfirstlane(more ? srdW[e] : nullW[e]);
#pragma clang loop unroll(full)
    for (int idx = 0; idx < 64; ++idx) {
      mf(idx, x1, w1);
#ifndef W4_ABL_NODMA
      if (idx >= W4_DB0 && (idx - W4_DB0) % W4_DBS == 0 && (idx - W4_DB0) / W4_DBS < 16)
        dma(t + 2, cur, (idx - W4_DB0) / W4_DBS, sX, sW);
#endif
#ifndef W4_ABL_NOREAD
      if (idx >= W4_RB0 && (idx - W4_RB0) % W4_RBS == 0 && (idx - W4_RB0) / W4_RBS < 16)
        read_frag(cur ^ 1, 0, (idx - W4_RB0) / W4_RBS, x0, w0);  // tile t+1 (garbage after the last)
#endif
    }
  };
#ifdef W4_STAMPS  // diagnostic build: per-wave cycles in phase A / the wait + barrier / phase B
  uint64_t cyc_a = 0, cyc_w = 0, cyc_b = 0, t_end = __builtin_amdgcn_s_memtime();
#endif
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
#pragma clang loop unroll(full)
    for (int idx = 0; idx < 64; ++idx) {  // phase A
      mf(idx, x0, w0);
#ifndef W4_ABL_NOREAD
      if (idx >= W4_RA0 && (idx - W4_RA0) % W4_RAS == 0 && (idx - W4_RA0) / W4_RAS < 16)
        read_frag(cur, 1, (idx - W4_RA0) / W4_RAS, x1, w1);
#endif
    }
#ifdef W4_STAMPS
    const uint64_t t_a = __builtin_amdgcn_s_memtime();
#endif
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
#ifdef W4_STAMPS
    const uint64_t t_w = __builtin_amdgcn_s_memtime();
    cyc_a += t_a - t_end, cyc_w += t_w - t_a;
#endif
    phase_b(t, cur);
#ifdef W4_STAMPS
    t_end = __builtin_amdgcn_s_memtime();
    cyc_b += t_end - t_w;
#endif
  }
#ifdef W4_STAMPS
  if (lane == 0 && blockIdx.x < 4096) {
    uint64_t* st = w4_stamps + (static_cast<size_t>(blockIdx.x) * 4 + wave) * 4;
    st[0] = cyc_a, st[1] = cyc_w, st[2] = cyc_b, st[3] = nk;
  }
#endif
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  // the last MFMAs' results are read by VALU / stores below: cover the MFMA D -> read hazard
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");

  // ---- epilogue: lane holds D[n = 4fq + e][m = fr] of block (i, j), value(i, j) ----
  auto epilogue = [&](auto value) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int m = m0 + wm * 128 + j * 16 + fr;
      if (m >= M) continue;
      if constexpr (EPI == EPI_SILU_MUL) {
#pragma unroll
        for (int i = 0; i < 8; i += 2) {  // (gate, up) block pairs of the same 16 features
          const int feat = (n0 >> 1) + wn * 64 + (i >> 1) * 16 + 4 * fq;
          const f32x4 g = value(i, j), u = value(i + 1, j);
          *reinterpret_cast<u16x4*>(C + static_cast<size_t>(m) * ldc + feat) =
              pack4(silu(g[0]) * u[0], silu(g[1]) * u[1], silu(g[2]) * u[2], silu(g[3]) * u[3]);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int n = n0 + wn * 128 + i * 16 + 4 * fq;
          if (n >= N) continue;
          f32x4 v = value(i, j);
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
          *reinterpret_cast<u16x4*>(C + static_cast<size_t>(m) * ldc + n) = pack4(v[0], v[1], v[2], v[3]);
        }
      }
    }
  };

  if (split_k == 1) {
    epilogue([&](int i, int j) { return acc[i][j]; });
    return;
  }
  // ---- split-K: every split stores its fp32 tile write-through (sc1); the last arriver sums
  // all the slabs (its own included) straight into the epilogue -- the accumulators die at
  // the store, so the reduction needs no second register copy of the tile
  float* slab = ws + static_cast<size_t>(tile) * split_k * (BM * BN);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(slab, 0, split_k * BM * BN * 4, 0x00020000);
  __syncthreads();  // every wave is past its last ds_read: smem is reusable as the flag slot
  int* flag = reinterpret_cast<int*>(smem);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int off = (split * (BM * BN) + ((wave * 8 + i) * 8 + j) * 256 + lane * 4) * 4;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs, off, 0, 16 /*sc1*/);
    }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int prev = __hip_atomic_fetch_add(&counters[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == split_k - 1;
    if (last) __hip_atomic_store(&counters[tile], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag[0] = last;
  }
  __syncthreads();
  if (!flag[0]) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  epilogue([&](int i, int j) {
    f32x4 sum = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int sp = 0; sp < split_k; ++sp) {
      const int off = (sp * (BM * BN) + ((wave * 8 + i) * 8 + j) * 256 + lane * 4) * 4;
      sum += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16 /*sc1*/));
    }
    return sum;
  });
}

template <int EPI>
int launch_w4(const void* x, const void* w, const void* bias, const void* res, void* c, float* ws, int* cnt, int M,
              int N, int K, int inter, int split_k, hipStream_t stream) {
  const int m_tiles = (M + BM - 1) / BM, n_tiles = (N + BN - 1) / BN;
  const int ldc = EPI == EPI_SILU_MUL ? inter : N;
  hipLaunchKernelGGL((gemm_w4_kernel<EPI>), dim3(m_tiles * n_tiles * split_k), dim3(256), 0, stream,
                     static_cast<const bf16_t*>(x), static_cast<const bf16_t*>(w), static_cast<const bf16_t*>(bias),
                     static_cast<const bf16_t*>(res), static_cast<bf16_t*>(c), ws, cnt, M, N, K, ldc, inter, m_tiles,
                     n_tiles, split_k);
  return BCG_CHECK_LAUNCH();
}

}  // namespace

#ifdef W4_STAMPS
// diagnostic build only: copy the per-wave cycle stamps of the last launch to the host
BCG_API int bcg_gemm_w4_stamps(void* host, int n) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(w4_stamps), sizeof(uint64_t) * n) == hipSuccess ? 0 : -1;
}
#endif

// Same contract as bcg_gemm_pp: epi 0 = store (+bias), 1 = silu(gate)*up into [M, inter],
// 2 = residual + acc.  K % 64 == 0, K/64 >= split_k; N % 16 == 0 (a partial last n-tile is
// masked); EPI 1: N == 2*inter, inter % 128 == 0.  split_k > 1: `ws` >= m_tiles*n_tiles*
// split_k*65536 floats, `counters` >= m_tiles*n_tiles zeroed ints (left zeroed).
BCG_API int bcg_gemm_w4(int epi, const void* x, const void* w, const void* bias, const void* residual, void* c,
                        void* ws, void* counters, int M, int N, int K, int inter, int split_k, hipStream_t stream) {
  if (M <= 0 || N <= 0 || N % 16 || K % BK || K <= 0 || split_k < 1 || K / BK < split_k) return -2;
  // 32-bit buffer offsets, rows up to a whole tile past the end included
  if (2ull * (M + BM) * K >= (1ull << 31) || 2ull * (N + BN) * K >= (1ull << 31)) return -2;
  if (split_k > 1 && (!ws || !counters)) return -2;
  float* wsf = static_cast<float*>(ws);
  int* cnt = static_cast<int*>(counters);
  switch (epi) {
    case EPI_STORE: return launch_w4<EPI_STORE>(x, w, bias, residual, c, wsf, cnt, M, N, K, inter, split_k, stream);
    case EPI_SILU_MUL:
      if (N != 2 * inter || inter % 128) return -2;
      return launch_w4<EPI_SILU_MUL>(x, w, nullptr, nullptr, c, wsf, cnt, M, N, K, inter, split_k, stream);
    case EPI_RESIDUAL:
      if (!residual) return -2;
      return launch_w4<EPI_RESIDUAL>(x, w, bias, residual, c, wsf, cnt, M, N, K, inter, split_k, stream);
    default: return -2;
  }
}
