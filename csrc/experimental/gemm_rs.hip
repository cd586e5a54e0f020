// 256 x 256 x 64 GEMM with REGISTER-staged operands, one wave per SIMD (gfx950).
//
// EXPERIMENTAL (tools-only build, tools/build_gemm_variants.sh): correct (the GPU GEMM tests
// passed with it registered as a tile configuration) but SLOWER than the LDS-DMA ping-pong
// kernel on every Qwen3-14B shape, 1.10-1.25 vs 1.23-1.28 PF/s at M = 16384 and far behind at
// the split-K decode shapes (profiles/r3_gemm_rs/).  PMC (profiles/r3_gemm_rs/summary_*.txt,
// down_proj 16384 x 5120 x 17408): MFMA pipe busy 46 % vs 60 %; the waves sit in issue stalls
// (SQ_WAIT_INST_ANY 63 % of wave cycles, LDS-issue stalls 13 %) and an LDS instruction costs
// 2.3x the ping-pong kernel's (SQ_ACTIVE_INST_LDS 156 M vs 67 M for the same instruction
// count): the 16 ds_write_b128 per K-tile that one wave per SIMD must issue are as expensive
// as the LDS-DMA pieces they replace, and no partner wave covers them.
//
//   C[M, N] = X[M, K] · W[N, K]^T            (bf16 in, fp32 accumulate, bf16 out)
//
// The third tile family beside gemm.hip (decode tiles) and gemm_pp.hip (256 x 256
// ping-pong): the same output tile and fused epilogues, fed differently.  gemm_pp moves
// every K-tile global -> LDS by LDS-DMA (`global_load_lds`, 1 KiB per wave-instruction);
// its ablations put the wall there: each piece holds its issuing wave for ~100 cycles and
// a CU takes in ~48 GB/s that way (PERF.md "Large shapes"), against the ~46 GB/s per CU a
// 1.5 PF/s 256 x 256 tile needs.  Here the operands take the ordinary vector-memory path
// (`buffer_load_dwordx4` into VGPRs, coalesced 128-B rows) and are written to LDS with
// `ds_write_b128` one K-tile later, the classic register-staged double buffer
// (cdna_hip_programming.md §6 Guideline 15, T14) -- affordable because each wave owns a
// whole SIMD (512 registers: 256 accumulators + fragments + one K-tile of staging).
//
// Structure
//   * workgroup = 4 waves, wave w owns the 128 x 128 output quadrant (w & 1, w >> 1):
//     8 x 8 blocks of v_mfma_f32_16x16x32_bf16 = 256 accumulator registers; per 64-deep
//     K-tile 128 MFMAs against 32 ds_read_b128 (half the LDS bytes per FLOP of a
//     128 x 64 wave tile) and 16 buffer loads + 16 LDS writes;
//   * LDS: two stages of A (256 X rows) + B (256 W rows) x 128 B = 128 KiB; the 16-B chunk
//     c of row r at c ^ ((r >> 1) & 7) (conflict-free fragment reads, as gemm.hip);
//   * per K-tile t (stage t & 1), ONE operation beside each MFMA (RS_* schedule below): the
//     k-step-1 fragment reads, tile t+1's LDS writes (in registers since the previous tile),
//     tile t+2's loads into the freed registers, one barrier, the first fragments of tile
//     t+1 -- the wave never stops issuing MFMAs for a burst of memory instructions;
//   * the operands are swapped in the MFMA (W fragment as A, X fragment as B) so a lane
//     holds 4 consecutive output columns of one row (8-B stores, gate/up pairs in one
//     lane), XCD-aware grouped tile order and last-arriver split-K, as gemm_pp.hip.
// SURVEY.md §2.3 K-GEMM-QKV/O/GU/D/LMH (the reference reaches these GEMMs inside vLLM,
// byzantine_consensus_game/vllm_agent.py:430).
#include "common.h"

#ifndef RS_GROUP_M
#define RS_GROUP_M 8  // m-tiles per tile-order group (L2 reuse of both operands at prefill M)
#endif
// K-tile schedule (MFMA index, 0..127, where each group of 16 operations starts): see the loop
#ifndef RS_R1
#define RS_R1 0
#endif
#ifndef RS_W
#define RS_W 48
#endif
#ifndef RS_L
#define RS_L 64
#endif
#ifndef RS_B
#define RS_B 96
#endif

namespace {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int A_BYTES = BM * 128, STAGE = A_BYTES + BN * 128;  // 64 KiB
enum Epilogue { EPI_STORE = 0, EPI_SILU_MUL = 1, EPI_RESIDUAL = 2 };

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float silu(float g) { return g / (1.f + __expf(-g)); }

// f32 -> bf16 by the hardware convert (v_cvt_pk_bf16_f32: round to nearest even, NaN kept):
// branch-free, unlike the bit-twiddling f2bf of common.h
__device__ __forceinline__ u16x4 pack4(float a, float b, float c, float d) {
  typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
  const bf16x4 v = {static_cast<__bf16>(a), static_cast<__bf16>(b), static_cast<__bf16>(c), static_cast<__bf16>(d)};
  return __builtin_bit_cast(u16x4, v);
}

template <int EPI>
__global__ __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_rs_kernel(
    const bf16_t* __restrict__ X, const bf16_t* __restrict__ W, const bf16_t* __restrict__ bias,
    const bf16_t* __restrict__ residual, bf16_t* __restrict__ C, float* __restrict__ ws,
    int* __restrict__ counters, int M, int N, int K, int ldc, int inter, int m_tiles, int n_tiles,
    int split_k) {
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * STAGE];

  // ---- XCD-aware order (bijective remap), grouped m-tiles, then (tile, k-split) ----
  const int nwg = m_tiles * n_tiles * split_k;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, rem = nwg & 7;
  const int r_id = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (bid >> 3);
  const int split = r_id % split_k;
  const int tile = r_id / split_k;
  const int grp = tile / (RS_GROUP_M * n_tiles), in_grp = tile % (RS_GROUP_M * n_tiles);
  const int gm = min(m_tiles - grp * RS_GROUP_M, RS_GROUP_M);
  const int m_tile = grp * RS_GROUP_M + in_grp % gm, n_tile = in_grp / gm;
  const int m0 = m_tile * BM, n0 = n_tile * BN;
  const int nk_all = K / BK;
  const int kt0 = split * nk_all / split_k;
  const int nk = (split + 1) * nk_all / split_k - kt0;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int fr = lane & 15, fq = lane >> 4;

  // ---- staging: thread tid moves chunk (tid & 7) of rows i*32 + (tid >> 3), i = 0..7, of
  // both operands.  Rows past M / N read zeros (buffer range check) and are never stored.
  const int r0 = tid >> 3, ch = tid & 7;
  const uint32_t row_bytes = static_cast<uint32_t>(K) * 2;
  const __amdgpu_buffer_rsrc_t rsX =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(X), 0, static_cast<uint32_t>(M) * row_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsW = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(W), 0, static_cast<uint32_t>(EPI == EPI_SILU_MUL ? 2 * inter : N) * row_bytes, 0x00020000);
  const uint32_t voffX = static_cast<uint32_t>(m0 + r0) * row_bytes + ch * 16;
  // W rows: plain n0 + i*32 + r0; SILU: 16-row blocks alternate gate / up of the same features,
  // so piece i of thread tid is row (r0 >> 4) * inter + n0/2 + i*16 + (r0 & 15)
  const uint32_t voffW = static_cast<uint32_t>(EPI == EPI_SILU_MUL ? (r0 >> 4) * inter + (n0 >> 1) + (r0 & 15)
                                                                   : n0 + r0) * row_bytes + ch * 16;
  const uint32_t strideW = (EPI == EPI_SILU_MUL ? 16u : 32u) * row_bytes;
  const uint32_t strideX = 32u * row_bytes;
  const int st_off = r0 * 128 + ((ch ^ ((r0 >> 1) & 7)) << 4);  // + i * 4096 (rows i*32+r0 share the swizzle)

  u32x4 stg[16];  // one K-tile: 8 X pieces, 8 W pieces
  auto load_tile = [&](int t) {
    const uint32_t k0b = static_cast<uint32_t>(kt0 + t) * (BK * 2);
#pragma unroll
    for (int i = 0; i < 8; ++i)
      stg[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsX, voffX + i * strideX, k0b, 0));
#pragma unroll
    for (int i = 0; i < 8; ++i)
      stg[8 + i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rsW, voffW + i * strideW, k0b, 0));
  };
  auto store_tile = [&](int stage) {
    unsigned char* base = smem + stage * STAGE + st_off;
#pragma unroll
    for (int i = 0; i < 8; ++i) *reinterpret_cast<u32x4*>(base + i * 4096) = stg[i];
#pragma unroll
    for (int i = 0; i < 8; ++i) *reinterpret_cast<u32x4*>(base + A_BYTES + i * 4096) = stg[8 + i];
  };

  f32x4 acc[8][8];  // [n-block][m-block]
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Fragments of a 32-deep k-step: fragment f < 8 is X block f (rows wm*128 + 16f + fr),
  // f >= 8 is W block f-8 (rows wn*128 + 16(f-8) + fr); chunk 4*s + fq, swizzled.
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
  // MFMA idx of a k-step (n-block idx >> 3, m-block idx & 7), accumulator pinned in AGPRs:
  // with the builtin, hipcc (ROCm 7.2) cycled this kernel's 256 accumulator registers through
  // a[0:3] around every MFMA (~470 v_accvgpr moves per K-tile).  "memory" keeps the source
  // order of the MFMAs and of the LDS / global accesses written between them (the
  // interleave below).  Operands come straight from ds_read (hipcc waits lgkmcnt before
  // the statement; no VALU-write -> MFMA-read hazard to pad); the D -> VALU-read hazard is
  // padded once after the main loop.
  auto mf = [&](int idx, const bf16x8 (&xf)[8], const bf16x8 (&wf)[8]) {
    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                 : "+a"(acc[idx >> 3][idx & 7])
                 : "v"(wf[idx >> 3]), "v"(xf[idx & 7])
                 : "memory");
  };
  auto barrier = [&]() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
  const uint32_t last_k0b = static_cast<uint32_t>(kt0 + nk - 1) * (BK * 2);

  // ---- prologue: tile 0 -> stage 0, tile 1 in registers, k-step 0 fragments of tile 0 ----
  bf16x8 x0[8], w0[8], x1[8], w1[8];
  load_tile(0);
  store_tile(0);
  load_tile(nk > 1 ? 1 : 0);
  barrier();
#pragma unroll
  for (int f = 0; f < 16; ++f) read_frag(0, 0, f, x0, w0);

  // Steady state, branch-free: the loads run one tile past the end (the last tile again) and
  // the last iteration writes / reads that copy into the free stage -- never used.  The 128
  // MFMAs of a K-tile (k-step 0: 0-63, k-step 1: 64-127) carry, one per MFMA:
  //   [RS_R1, +16)  the k-step-1 fragment reads of tile t (stage cur)        RS_R1 + 16 <= 64
  //   [RS_W, +16)   the LDS writes of tile t+1 (registers -> stage cur^1)
  //   [RS_L, +16)   the global loads of tile t+2 (into the registers just written out)
  //   RS_B          lgkmcnt(0) + barrier: tile t+1 visible; stage cur's reads retired everywhere
  //   [RS_B, +16)   the k-step-0 fragment reads of tile t+1                  RS_B >= 64
  static_assert(RS_R1 + 16 <= 64 && RS_W + 16 <= RS_L && RS_L + 16 <= 128 && RS_W + 16 <= RS_B &&
                    RS_B >= 64 && RS_B + 16 <= 128, "K-tile schedule");
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    unsigned char* st_base = smem + (cur ^ 1) * STAGE + st_off;
    const uint32_t k0b = min(static_cast<uint32_t>(kt0 + t + 2) * (BK * 2), last_k0b);
#pragma clang loop unroll(full)  // every index static: a rolled loop puts acc in scratch (see mf)
    for (int idx = 0; idx < 128; ++idx) {
      if (idx == RS_B) barrier();
      if (idx < 64)
        mf(idx, x0, w0);
      else
        mf(idx - 64, x1, w1);
      if (idx >= RS_R1 && idx < RS_R1 + 16) read_frag(cur, 1, idx - RS_R1, x1, w1);
      if (idx >= RS_W && idx < RS_W + 16) {
        const int q = idx - RS_W;
        *reinterpret_cast<u32x4*>(st_base + (q & 7) * 4096 + (q < 8 ? 0 : A_BYTES)) = stg[q];
      }
      if (idx >= RS_L && idx < RS_L + 16) {
        const int q = idx - RS_L;
        stg[q] = __builtin_bit_cast(
            u32x4, q < 8 ? __builtin_amdgcn_raw_buffer_load_b128(rsX, voffX + q * strideX, k0b, 0)
                         : __builtin_amdgcn_raw_buffer_load_b128(rsW, voffW + (q - 8) * strideW, k0b, 0));
      }
      if (idx >= RS_B && idx < RS_B + 16) read_frag(cur ^ 1, 0, idx - RS_B, x0, w0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // the surplus loads / reads

  // the last MFMAs' results are read by VALU / stores below: cover the MFMA D -> read hazard
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");

  // ---- split-K: partial tiles -> workspace (write-through); the last arriver reduces ----
  if (split_k > 1) {
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
    for (int sp = 0; sp < split_k; ++sp) {
      if (sp == split) continue;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int off = (sp * (BM * BN) + ((wave * 8 + i) * 8 + j) * 256 + lane * 4) * 4;
          acc[i][j] += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16 /*sc1*/));
        }
    }
  }

  // ---- epilogue: lane holds D[n = 4fq + e][m = fr] of block (i, j) ----
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int m = m0 + wm * 128 + j * 16 + fr;
    if (m >= M) continue;
    if constexpr (EPI == EPI_SILU_MUL) {
#pragma unroll
      for (int i = 0; i < 8; i += 2) {  // (gate, up) block pairs of the same 16 features
        const int feat = (n0 >> 1) + wn * 64 + (i >> 1) * 16 + 4 * fq;
        const f32x4 g = acc[i][j], u = acc[i + 1][j];
        *reinterpret_cast<u16x4*>(C + static_cast<size_t>(m) * ldc + feat) =
            pack4(silu(g[0]) * u[0], silu(g[1]) * u[1], silu(g[2]) * u[2], silu(g[3]) * u[3]);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int n = n0 + wn * 128 + i * 16 + 4 * fq;
        if (n >= N) continue;
        float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
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
}

template <int EPI>
int launch_rs(const void* x, const void* w, const void* bias, const void* res, void* c, float* ws, int* cnt, int M,
              int N, int K, int inter, int split_k, hipStream_t stream) {
  const int m_tiles = (M + BM - 1) / BM, n_tiles = (N + BN - 1) / BN;
  const int ldc = EPI == EPI_SILU_MUL ? inter : N;
  hipLaunchKernelGGL((gemm_rs_kernel<EPI>), dim3(m_tiles * n_tiles * split_k), dim3(256), 0, stream,
                     static_cast<const bf16_t*>(x), static_cast<const bf16_t*>(w), static_cast<const bf16_t*>(bias),
                     static_cast<const bf16_t*>(res), static_cast<bf16_t*>(c), ws, cnt, M, N, K, ldc, inter, m_tiles,
                     n_tiles, split_k);
  return BCG_CHECK_LAUNCH();
}

}  // namespace

// Same contract as bcg_gemm_pp: epi 0 = store (+bias), 1 = silu(gate)*up into [M, inter],
// 2 = residual + acc.  K % 64 == 0, K/64 >= split_k; N % 16 == 0 (a partial last n-tile is
// masked); EPI 1: N == 2*inter, inter % 128 == 0.  split_k > 1: `ws` >= m_tiles*n_tiles*
// split_k*65536 floats, `counters` >= m_tiles*n_tiles zeroed ints (left zeroed).
BCG_API int bcg_gemm_rs(int epi, const void* x, const void* w, const void* bias, const void* residual, void* c,
                        void* ws, void* counters, int M, int N, int K, int inter, int split_k, hipStream_t stream) {
  if (M <= 0 || N <= 0 || N % 16 || K % BK || K <= 0 || split_k < 1 || K / BK < split_k) return -2;
  if (2ull * (M + BM) * K >= (1ull << 32) || 2ull * (N + BN) * K >= (1ull << 32)) return -2;  // 32-bit offsets
  if (split_k > 1 && (!ws || !counters)) return -2;
  float* wsf = static_cast<float*>(ws);
  int* cnt = static_cast<int*>(counters);
  switch (epi) {
    case EPI_STORE: return launch_rs<EPI_STORE>(x, w, bias, residual, c, wsf, cnt, M, N, K, inter, split_k, stream);
    case EPI_SILU_MUL:
      if (N != 2 * inter || inter % 128) return -2;
      return launch_rs<EPI_SILU_MUL>(x, w, nullptr, nullptr, c, wsf, cnt, M, N, K, inter, split_k, stream);
    case EPI_RESIDUAL:
      if (!residual) return -2;
      return launch_rs<EPI_RESIDUAL>(x, w, bias, residual, c, wsf, cnt, M, N, K, inter, split_k, stream);
    default: return -2;
  }
}
