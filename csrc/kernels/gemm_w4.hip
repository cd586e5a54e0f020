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
// Schedule (one K-tile t; LDS = a ring of five 32-KiB slots, tile t's X and W halves in slots
// 2t and 2t+1 mod 5; every index static):
//   phase A: 64 MFMAs of k-step 0 (fragments x0/w0 in registers)
//            || 16 ds_read_b128 of k-step 1 of tile t -> x1/w1
//            || 8 LDS-DMA pieces of X(t+2) into the slot W(t-1) freed
//            then  s_waitcnt vmcnt(8) lgkmcnt(0); s_barrier  (tile t+1 landed, X(t+2) may fly)
//   phase B: 64 MFMAs of k-step 1 (x1/w1)
//            || 8 LDS-DMA pieces of W(t+2)
//            || 16 ds_read_b128 of k-step 0 of tile t+1 -> x0/w0
// RAW: a piece is waited for by every wave (counted vmcnt) before the barrier that precedes its
//      first read.  WAR: a slot is refilled only after the barrier that follows its last reads
//      (lgkmcnt(0) before that barrier).  Odd waves issue their pieces half a stride later.
// One barrier per K-tile, a piece has 1.5 phases (~1500 cycles) to land.
//
// LDS: rows of 128 B (64 bf16 of K), the 16-B chunk c of row r at c ^ ((r >> 1) & 7): the
// fragment ds_read_b128s are conflict-free (gemm.hip); LDS-DMA writes lane-linearly, so the
// swizzle is applied to each lane's SOURCE chunk.  Operands swapped in the MFMA (W fragment
// as A) so a lane holds 4 consecutive output columns of one row.  XCD-aware grouped tile
// order and last-arriver split-K as gemm_pp.hip; the same host contract (bcg_gemm_w4).
#include <algorithm>
#include <type_traits>

#include "common.h"

#ifndef W4_GROUP_M_F8
#define W4_GROUP_M_F8 4  // (fp8: 4 measured +2-15 % over 8 on Mistral-22B prefill shapes, profiles/r4_gemm_w4)
#endif
#ifndef W4_GROUP_M
#define W4_GROUP_M 8  // m-tiles per tile-order group (L2 reuse of both operands)
#endif
// schedule knobs: first MFMA slot and slot stride of each memory-op stream (W4_SLOTS per phase)
#define W4_SLOTS 64
// Defaults (measured, profiles/r4_gemm_w4/): the five-slot ring; phase A: the 16 k-step-1
// reads in its first half, X(t+2)'s 8 pieces in its second; phase B: W(t+2)'s 8 pieces every
// 8th slot, the 16 next-tile reads every 4th.
#ifndef W4_RA0
#define W4_RA0 0  // phase A: k-step-1 reads
#endif
#ifndef W4_RAS
#define W4_RAS (W4_SLOTS / 32)
#endif
#ifndef W4_DA0
#define W4_DA0 (W4_SLOTS / 2 + 1)  // RING5 phase A: LDS-DMA pieces of X(t+2)
#endif
#ifndef W4_DAS
#define W4_DAS (W4_SLOTS / 16)
#endif
#ifndef W4_DB0
#define W4_DB0 0  // phase B: LDS-DMA pieces
#endif
#ifndef W4_DBS
#define W4_DBS (W4_SLOTS / 8)
#endif
#ifndef W4_RB0
#define W4_RB0 (W4_SLOTS / 32)  // phase B: k-step-0 reads of the next tile
#endif
#ifndef W4_RBS
#define W4_RBS (W4_SLOTS / 16)
#endif
#define W4_NPB 8  // pieces issued in phase B (W(t+2)); phase A issues X(t+2)'s 8
#ifndef W4_PERSIST
#define W4_PERSIST 1  // one workgroup per CU streaming its tiles (split_k == 1; profiles/r4_gemm_w4)
#endif
static_assert(W4_DA0 + 7 * W4_DAS < W4_SLOTS, "phase A's X pieces fit the phase");

namespace {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int W4_COUNTERS = 65536;  // the caller's arrival-counter array (one per tile)
constexpr int A_BYTES = BM * 128;  // one operand's K-tile: 256 rows of 128 B
enum Epilogue { EPI_STORE = 0, EPI_SILU_MUL = 1, EPI_RESIDUAL = 2 };
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef int i32x8 __attribute__((ext_vector_type(8)));

static_assert(W4_RA0 + 15 * W4_RAS < W4_SLOTS && W4_DB0 + (W4_NPB - 1) * W4_DBS < W4_SLOTS &&
                  W4_RB0 + 15 * W4_RBS < W4_SLOTS,
              "each stream fits its phase");
typedef float f32x16 __attribute__((ext_vector_type(16)));

// g * sigmoid(g) with the hardware reciprocal (1 ulp; a true division expands to ~10
// instructions with mode switches per element in the epilogue)
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

// Staggered schedules (W4_STAGGER): the odd waves issue their pieces half a stride later than
// the even waves, so the CU's four waves do not send their LDS-DMA in lock step (the same
// device as the two loop bodies, selected by a SIMD-id bit, of hipBLASLt's MT256x256 kernel).
struct SchedMain {
  static constexpr int RA0 = W4_RA0, RAS = W4_RAS, DA0 = W4_DA0, DAS = W4_DAS, DB0 = W4_DB0, DBS = W4_DBS,
                       RB0 = W4_RB0, RBS = W4_RBS;
};
struct SchedAlt {
  static constexpr int RA0 = W4_RA0, RAS = W4_RAS, DA0 = W4_DA0 + W4_DAS / 2, DAS = W4_DAS,
                       DB0 = W4_DB0 + W4_DBS / 2, DBS = W4_DBS, RB0 = W4_RB0, RBS = W4_RBS;
  static_assert(DA0 + 7 * DAS < W4_SLOTS && DB0 + (W4_NPB - 1) * DBS < W4_SLOTS, "staggered schedule");
};
// fp8 (e4m3) form: a K-tile is 128 elements in the same 128-B rows; each phase = one 64-deep
// k-step = 16 v_mfma_scale_f32_32x32x64_f8f6f4 (the cycles of 64 bf16 16x16x32), so the same
// 16 reads and 8 pieces per phase serve twice the FLOPs.
#ifndef W4F8_DA0
#define W4F8_DA0 8
#endif
#ifndef W4F8_DB0
#define W4F8_DB0 0
#endif
struct SchedF8 {
  static constexpr int RA0 = 0, RAS = 1, DA0 = W4F8_DA0, DAS = 1, DB0 = W4F8_DB0, DBS = 2, RB0 = 0, RBS = 1;
  static_assert(DA0 + 7 * DAS < 16 && DB0 + 7 * DBS < 16, "fp8 schedule");
};
struct SchedF8Alt {
  static constexpr int RA0 = 0, RAS = 1, DA0 = W4F8_DA0 - 1, DAS = 1, DB0 = W4F8_DB0 + 1, DBS = 2, RB0 = 0, RBS = 1;
};

#ifdef W4_STAMPS
// [workgroup][wave][phase A, wait, phase B, K-tiles, epilogues, kernel total, items, -]
__device__ uint64_t w4_stamps[1 << 17];
#endif

// F8: e4m3 operands with v_mfma_scale_f32_32x32x64_f8f6f4 (unit E8M0 block scales; x_scale[m] *
// w_scale[n] applied in the epilogue)
template <int EPI, bool F8 = false>
__global__ __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm_w4_kernel(
    const void* __restrict__ Xv, const void* __restrict__ Wv, const bf16_t* __restrict__ bias,
    const bf16_t* __restrict__ residual, bf16_t* __restrict__ C, float* __restrict__ ws,
    int* __restrict__ counters, int M, int N, int K, int ldc, int inter, int m_tiles, int n_tiles,
    int split_k, const float* __restrict__ x_scale, const float* __restrict__ w_scale) {
  static_assert(!F8 || EPI != EPI_SILU_MUL, "fp8: store / residual epilogues");
  constexpr bool L32 = F8;                             // 32x32 accumulator layout
  constexpr int SLOTS = F8 ? 16 : W4_SLOTS;            // MFMAs per phase
  constexpr int ESZ = F8 ? 1 : 2;                      // bytes per element
  const unsigned char* X = static_cast<const unsigned char*>(Xv);
  const unsigned char* W = static_cast<const unsigned char*>(Wv);
  // ONE shared array (cdna_hip_programming.md "Projection GEMM" item 4a)
  __shared__ __attribute__((aligned(1024))) unsigned char smem[5 * A_BYTES];
  // LDS byte offset of tile t's X (part 0) or W (part 1) half: a ring of five 32-KiB slots, tile
  // t in slots 2t, 2t+1 (mod 5)
  auto slot_off = [](int t, int part) -> uint32_t { return static_cast<uint32_t>((2 * t + part) % 5) * A_BYTES; };

  // ---- work items.  split_k >= 1: nwg = tiles x k-splits.  A persistent launch (gridDim.x <
  // nwg, split_k == 1 only) gives workgroup b the items b, b + G, b + 2G, ...: one continuous
  // stream of K-tiles in which the next item's first tiles are already in flight while this
  // item's epilogue runs.  Item -> tile: XCD-aware bijective remap (item i runs on XCD i % 8 when
  // G % 8 == 0, so each XCD's CUs walk one contiguous range of remapped ids), grouped m-tiles,
  // then (tile, k-split).
  // split_k == 0: stream-K.  The tiles x K-tiles units are cut into G equal contiguous ranges;
  // logical workgroup r (XCD-grouped: the workgroups of one XCD own one contiguous eighth of
  // the units) streams range r -- a partial first tile, whole tiles, a partial last tile.
  // Whole tiles take the ordinary in-stream epilogue; a partial segment stores its fp32 part
  // (per wave, write-through) and the workgroup that arrives last for that tile adds every
  // segment's part after its stream and runs the epilogue -- nobody waits on another workgroup.
  // The tile quantisation of decode-size M goes away (gate_up at 704 rows: 408 tiles = 1.6 per
  // CU instead of two rounds).
  const bool sk = split_k == 0;
  const int nsplit = sk ? 1 : split_k;
  const int tiles = m_tiles * n_tiles;
  const int nwg = tiles * nsplit;
  const int G = gridDim.x;
  const int nk_all = K / (128 / ESZ);  // K-tiles of 128 B per row
  int r_wg = blockIdx.x;               // stream-K: the logical workgroup (bijective XCD grouping)
  if (sk) {
    const int b = blockIdx.x, xcd = b & 7, q = G >> 3, rem = G & 7;
    r_wg = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (b >> 3);
  }
  // (32-bit: the host keeps tiles x nk_all x G below 2^31)
  auto sk_u0 = [&](int r) { return static_cast<int>(static_cast<uint32_t>(r) * (tiles * nk_all) / G); };
  const int u0 = sk ? sk_u0(r_wg) : 0, u1 = sk ? sk_u0(r_wg + 1) : 0;
  const int T0 = u0 / nk_all;
  const int n_items = sk ? (u1 > u0 ? (u1 - 1) / nk_all - T0 + 1 : 0)
                         : (nwg - 1 - static_cast<int>(blockIdx.x)) / G + 1;
  struct Geo {
    int m0, n0, tile, split, k0, nk;  // output corner, tile id, k-split, first K-tile and K-tiles of the item
  };
  auto tile_geo = [&](Geo& g) {
    constexpr int GM = F8 ? W4_GROUP_M_F8 : W4_GROUP_M;
    const int grp = g.tile / (GM * n_tiles), in_grp = g.tile % (GM * n_tiles);
    const int gm = min(m_tiles - grp * GM, GM);
    g.m0 = (grp * GM + in_grp % gm) * BM;
    g.n0 = (in_grp / gm) * BN;
  };
  auto geo = [&](int j) {
    Geo g;
    if (sk) {
      g.tile = T0 + j;
      g.split = 0;
      const int s0 = max(u0, g.tile * nk_all), e0 = min(u1, (g.tile + 1) * nk_all);
      g.k0 = s0 - g.tile * nk_all;
      g.nk = e0 - s0;
    } else {
      const int i = blockIdx.x + j * G;
      const int xcd = i & 7, q = nwg >> 3, rem = nwg & 7;
      const int r_id = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (i >> 3);
      g.split = r_id % split_k;
      g.tile = r_id / split_k;
      g.k0 = g.split * nk_all / split_k;
      g.nk = (g.split + 1) * nk_all / split_k - g.k0;
    }
    tile_geo(g);
    return g;
  };
  Geo gc = geo(0);                                     // the item whose accumulators are live
  const int total = sk ? u1 - u0 : n_items * gc.nk;    // K-tiles of the stream

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1;
  const int fr = lane & 15, fq = lane >> 4;

  // ---- LDS-DMA pieces: piece i (0..7) of wave w fills stage rows 32 i + 8 w + (lane >> 3),
  // physical chunk lane & 7 <- logical chunk (lane & 7) ^ ((4 w + (lane >> 4)) & 7).  Rows past
  // M / N fall outside the descriptor's range and read zeros (never stored).  Each item's
  // descriptors start at its first X / W row, so the lane offsets are the same for every item.
  const uint32_t row_bytes = static_cast<uint32_t>(K) * ESZ;
  const int prow = 8 * wave + (lane >> 3);
  const int pch = ((lane & 7) ^ ((4 * wave + (lane >> 4)) & 7)) * 16;
  const int w_rows = EPI == EPI_SILU_MUL ? 2 * inter : N;
  auto item_srd = [&](const Geo& g, i32x4& sX, i32x4& sW) {
    const int wr0 = EPI == EPI_SILU_MUL ? (g.n0 >> 1) : g.n0;
    sX = make_srd(X + static_cast<size_t>(g.m0) * row_bytes, static_cast<uint32_t>(M - g.m0) * row_bytes);
    sW = make_srd(W + static_cast<size_t>(wr0) * row_bytes, static_cast<uint32_t>(w_rows - wr0) * row_bytes);
  };
  const uint32_t voffX = static_cast<uint32_t>(prow) * row_bytes + pch;
  // SILU: 16-row blocks of the tile alternate gate / up of the same 16 features, so stage row
  // 32 i + r (r < 32) holds W row (r >> 4) * inter + n0/2 + 16 i + (r & 15)
  const uint32_t voffW =
      static_cast<uint32_t>(EPI == EPI_SILU_MUL ? (wave >> 1) * inter + (prow & 15) : prow) * row_bytes + pch;
  const uint32_t strideX = 32u * row_bytes;
  const uint32_t strideW = (EPI == EPI_SILU_MUL ? 16u : 32u) * row_bytes;
  // the row part of a piece's offset stays in the VGPR offset: only that is range-checked
  // (the SGPR offset carries the K-tile)
  uint32_t vX[8], vW[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) vX[i] = voffX + i * strideX, vW[i] = voffW + i * strideW;
  const uint32_t lds_base = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(smem));
  // piece q (0..15) of stream tile t: q < 8 X piece q, else W piece q - 8
  auto dma_m0 = [&](int t, int q) {
    return __builtin_amdgcn_readfirstlane(lds_base + slot_off(t, q >= 8) + (q & 7) * 4096 + wave * 1024);
  };
  // DMA cursor: stream tile t + 2 is K-tile dk0 + ktd of item jd, whose descriptors are dX / dW
  int jd = 0, ktd = 0, dk0 = gc.k0, dnk = gc.nk;
  // stream tile t = K-tile kt of the DMA cursor's item: M0 write + piece in one statement
  auto dma = [&](int t, int kt, int q, const i32x4& sX, const i32x4& sW) {
    const uint32_t kb = static_cast<uint32_t>(dk0 + kt) * (BK * 2);
    const bool isx = q < 8;
    const int i = q & 7;
    const uint32_t soff = __builtin_amdgcn_readfirstlane(kb);
    const uint32_t m0v = dma_m0(t, q);
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

  // ---- fragments of one phase (32 of the K-tile's 64; half s = 0: chunks 0-3, 1: chunks 4-7):
  //   16x16x32: block f < 8 = X rows wm*128 + 16 f + fr, f >= 8 = W rows wn*128 + 16 (f-8) + fr,
  //             chunk 4 s + fq;  lane -> swizzle (fr >> 1) & 7
  //   32x32x16: f < 8 = X k-step f >> 2 (16 deep), rows wm*128 + 32 (f & 3) + (lane & 31);
  //             f >= 8 = the same for W;  chunk 4 s + 2 ks + (lane >> 5); swizzle ((lane & 31) >> 1) & 7
  const int r_lane = L32 ? (lane & 31) : fr;
  const int rd_sw = (r_lane >> 1) & 7;
  const int rdA = (wm * 128 + r_lane) * 128, rdB = (wn * 128 + r_lane) * 128;
  auto read_frag = [&](int t, int s, int f, bf16x8 (&xf)[8], bf16x8 (&wf)[8]) {
    int off = slot_off(t, f >= 8) + (f < 8 ? rdA : rdB);
    if constexpr (F8) {  // block (f >> 1) & 3, 16-B chunk f & 1 of the lane's 32 k (k = 32 (lane >> 5) + ...)
      const int blk = (f >> 1) & 3;
      off += (((4 * s + 2 * (lane >> 5) + (f & 1)) ^ rd_sw) << 4) + blk * 4096;
    } else {
      off += (((4 * s + fq) ^ rd_sw) << 4) + (f & 7) * 2048;
    }
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(smem + off);
    if (f < 8)
      xf[f] = v;
    else
      wf[f - 8] = v;
  };

  // accumulators, pinned in AGPRs by the asm MFMA below: [n-block][m-block]
  using Acc = std::conditional_t<L32, f32x16[4][4], f32x4[8][8]>;
  constexpr int NB = L32 ? 4 : 8;
  Acc acc;
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = 0.f;
  // "memory" keeps the MFMAs in source order with the LDS reads and DMA issued between them;
  // the builtin form lets hipcc cycle the accumulators through a few AGPRs (gemm_rs.hip)
  const int e8m0_one = 127;  // E8M0 block scale 1.0 (VGPR operand of the scaled MFMA)
  auto mf = [&](int idx, const bf16x8 (&xf)[8], const bf16x8 (&wf)[8]) {
    if constexpr (F8) {  // idx = nb * 4 + mb; a block's operand = its two 16-B chunks
      const int nb = idx >> 2, mb = idx & 3;
      const i32x8 a = __builtin_shufflevector(__builtin_bit_cast(i32x4, wf[2 * nb]),
                                              __builtin_bit_cast(i32x4, wf[2 * nb + 1]), 0, 1, 2, 3, 4, 5, 6, 7);
      const i32x8 b = __builtin_shufflevector(__builtin_bit_cast(i32x4, xf[2 * mb]),
                                              __builtin_bit_cast(i32x4, xf[2 * mb + 1]), 0, 1, 2, 3, 4, 5, 6, 7);
      asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, %0, %3, %3 op_sel_hi:[0,0,0]"
                   : "+a"(acc[nb][mb])
                   : "v"(a), "v"(b), "v"(e8m0_one)
                   : "memory");
    } else {
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                   : "+a"(acc[idx >> 3][idx & 7])
                   : "v"(wf[idx >> 3]), "v"(xf[idx & 7])
                   : "memory");
    }
  };

  bf16x8 x0[8], w0[8], x1[8], w1[8];
  i32x4 dX, dW;
  item_srd(gc, dX, dW);
  i32x4 nullX = dX, nullW = dW;  // zero-range descriptors: pieces past the stream's last tile
  nullX[2] = 0, nullW[2] = 0;
  auto advance = [&]() {
    if (++ktd == dnk) {
      ktd = 0;
      if (++jd < n_items) {
        const Geo g = geo(jd);
        item_srd(g, dX, dW);
        dk0 = g.k0, dnk = g.nk;
      }
    }
  };
  // ---- prologue: stream tiles 0 and 1 in flight, tile 0 landed, k-step 0 of tile 0 in registers ----
#pragma unroll
  for (int q = 0; q < 16; ++q) dma(0, 0, q, dX, dW);
  advance();
  if (total > 1) {
#pragma unroll
    for (int q = 0; q < 16; ++q) dma(1, ktd, q, dX, dW);
    asm volatile("s_waitcnt vmcnt(16)\n\ts_barrier" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  }
#pragma unroll
  for (int f = 0; f < 16; ++f) read_frag(0, 0, f, x0, w0);

  // ---- epilogue of item g.  The tile is seen as [n-group][m-block] quads of 4 consecutive output
  // columns (n) of one row (m) per lane: q = quad(i, j) with i over 32 n-groups, j over NB m-blocks.
  //   16x16x32: block (nb, mb) lane: D[n = 16 nb + 4 fq + e][m = 16 mb + fr];  i = nb
  //   32x32x16: block (nb, mb) lane: D[n = 32 nb + 8 g + 4 (lane >> 5) + e][m = 32 mb + (lane & 31)],
  //             registers 4 g + e;  i = 4 nb + g (g = 0..3)
  // value(nb, mb) returns the block's registers (accumulators, or the split-K slab sum).
  auto epilogue = [&](const Geo& geo_c, auto value) {
    constexpr int MB = L32 ? 32 : 16;
    constexpr int NG = L32 ? 4 : 1;  // quads per block
    // the lane index re-enters here through an opaque move: the epilogue's per-lane address
    // math cannot be hoisted out of the K-loop (it would hold ~100 VGPRs across it and spill)
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int fr = ln & 15, fq = ln >> 4;
    const int ml = L32 ? (ln & 31) : fr;
    const int m0 = geo_c.m0, n0 = geo_c.n0;
    auto row = [&](int j) { return m0 + wm * 128 + j * MB + ml; };
    auto st4 = [&](bf16_t* p, u16x4 v) {
      *reinterpret_cast<u16x4*>(p) = v;
    };
    if constexpr (!L32) {
      // 16x16 layout, buffer-addressed, 16-B accesses.  A store costs per cache line it touches
      // (stamps: ~300 cycles a 16-row x 8-B store, the same for 16 rows x 16 B), so two
      // neighbouring quads (4 columns of blocks 2p and 2p+1) are turned into 8 contiguous
      // columns per lane by one v_permlane16_swap per value: afterwards lane row fq holds
      // block 2p + (fq & 1), columns 8 (fq >> 1) .. +7 -- half the stores and loads.
      // Offsets are bytes from the item's output corner (C + m0 ldc + its first column): rows
      // past M fall outside the descriptor's range (stores dropped, loads 0), a column past N
      // gets an offset past every range -- no per-quad branch, no 64-bit address math.  The whole
      // offset (m-block j's rows included) rides in the VGPR: only that part is range-checked (an
      // SGPR offset is added after the check), and the host bounds (M + 256) * ldc * 2 below
      // 2^31 so a masked column's 0x80000000 + offset never wraps into range.
      constexpr bool SILU = EPI == EPI_SILU_MUL;
      constexpr int NP = SILU ? NB / 4 : NB / 2;  // 8-column groups per m-block per lane
      constexpr int JG = 1;                       // m-blocks per residual batch
      const uint32_t ldb = static_cast<uint32_t>(ldc) * 2;
      const int c0 = SILU ? (n0 >> 1) : n0;
      const uint32_t range = static_cast<uint32_t>(M - m0) * ldb;
      const auto rc = __builtin_amdgcn_make_buffer_rsrc(C + static_cast<size_t>(m0) * ldc + c0, 0, range, 0x00020000);
      const uint32_t rowv = static_cast<uint32_t>(wm * 128 + fr) * ldb;
      uint32_t colv[NP];
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const int cl = (SILU ? wn * 64 : wn * 128) + (2 * p + (fq & 1)) * 16 + (fq >> 1) * 8;
        colv[p] = SILU || n0 + cl < N ? static_cast<uint32_t>(cl) * 2 : 0x80000000u;
      }
      // lane-pair swap: a = 4 columns of the even quad, b = of the odd one -> o = 8 columns
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
        __builtin_amdgcn_raw_buffer_store_b128(pack8(o), rc, rowv + colv[p] + static_cast<uint32_t>(j * MB) * ldb, 0, 0);
      };
      if constexpr (SILU) {
#pragma unroll
        for (int j = 0; j < NB; ++j) {
#pragma unroll
          for (int p = 0; p < NP; ++p) {
            // 16-row blocks of the tile alternate gate / up of the same 16 features: output quad
            // q = blocks 2q (gate) and 2q + 1 (up); the pair p = quads 2p, 2p + 1
            float h[2][4];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
              const auto g = value(4 * p + 2 * k, j), u = value(4 * p + 2 * k + 1, j);
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
        // residual groups (8 bf16 per lane): batches of JG m-blocks, the next batch loaded
        // before this one is used
        u32x4 rq[2][JG][NP];
        auto load_rq = [&](int bf, int j0) {
          if constexpr (EPI == EPI_RESIDUAL) {
#pragma unroll
            for (int jj = 0; jj < JG; ++jj)
#pragma unroll
              for (int p = 0; p < NP; ++p)
                rq[bf][jj][p] = __builtin_amdgcn_raw_buffer_load_b128(
                    rr_rs, rowv + colv[p] + static_cast<uint32_t>((j0 + jj) * MB) * ldb, 0, 0);
          }
        };
        // one body per bias case (a uniform branch here, not one per quad); the bias groups
        // are widened to fp32 once per item
        auto body = [&](auto has_bias) {
          constexpr bool HB = decltype(has_bias)::value;
          u32x4 bq[HB ? NP : 1];  // 8 bf16 per group, widened where used
          if constexpr (HB) {
            const auto rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(bias + n0), 0,
                                                              static_cast<uint32_t>(N - n0) * 2, 0x00020000);
#pragma unroll
            for (int p = 0; p < NP; ++p) bq[p] = __builtin_amdgcn_raw_buffer_load_b128(rb, colv[p], 0, 0);
          }
          load_rq(0, 0);
#pragma unroll
          for (int j0 = 0; j0 < NB; j0 += JG) {
            const int bf = (j0 / JG) & 1;
            if (j0 + JG < NB) load_rq(bf ^ 1, j0 + JG);
#pragma unroll
            for (int jj = 0; jj < JG; ++jj)
#pragma unroll
              for (int p = 0; p < NP; ++p) {
                const auto a = value(2 * p, j0 + jj), b = value(2 * p + 1, j0 + jj);
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
                    const uint32_t w = rq[bf][jj][p][e >> 1];
                    o[e] += __uint_as_float((e & 1) ? (w & 0xffff0000u) : (w << 16));
                  }
                }
                store8(j0 + jj, p, o);
              }
            __builtin_amdgcn_sched_barrier(0);
          }
        };
        if (bias != nullptr)
          body(std::true_type{});
        else
          body(std::false_type{});
      }
      return;
    }
    if constexpr (EPI != EPI_SILU_MUL) {  // (the 32x32 layout is fp8's: store / residual only)
      // batches of JG m-blocks; the residual quads of the next batch are loaded before this
      // batch is computed (one HBM round trip per batch, overlapped, instead of one per quad)
      constexpr int JG = L32 ? 1 : 2;
      constexpr int NQ = NB * NG;  // quads per m-block per lane
      auto col = [&](int q) {
        const int nb = q / NG, g = q % NG;
        return n0 + wn * 128 + (L32 ? nb * 32 + 8 * g + 4 * (ln >> 5) : nb * 16 + 4 * fq);
      };
      // Every load is unconditional (addresses clamped into the tensor) and always consumed; only
      // the stores are masked.  A load whose result a masked path skipped would still be pending
      // at the K-loop's back edge, and hipcc's wait for it there (vmcnt(0) at the top of every
      // K-tile) would drain the LDS-DMA pieces in flight.
      auto mcl = [&](int m) { return m < M ? m : M - 1; };
      auto ncl = [&](int n) { return n < N ? n : N - 4; };
      u16x4 rr[2][JG][NQ];
      auto load_batch = [&](int bf, int j0) {
        if constexpr (EPI == EPI_RESIDUAL) {
#pragma unroll
          for (int jj = 0; jj < JG; ++jj)
#pragma unroll
            for (int q = 0; q < NQ; ++q)
              rr[bf][jj][q] = *reinterpret_cast<const u16x4*>(residual + static_cast<size_t>(mcl(row(j0 + jj))) * ldc +
                                                             ncl(col(q)));
        }
      };
      if constexpr (F8) {
        // fp8 (32x32 blocks): lane (r = lane & 31, h = lane >> 5) holds, per block and quad g,
        // columns 8 g + 4 h .. +3 of row r.  Scales go on per quad, then one v_permlane32_swap
        // per value turns quads g, g + 1 (g = 0, 2) into 8 contiguous columns per lane (h = 0:
        // 8 g .., h = 1: 8 (g + 1) ..): 16-B stores and loads, half the instructions (a store
        // costs per row it touches).  Buffer addressing as the 16x16 path; the residual and bias
        // descriptors have a zero range when unused (loads return 0).
        const int h = ln >> 5;
        const uint32_t ldb = static_cast<uint32_t>(ldc) * 2;
        const uint32_t range = static_cast<uint32_t>(M - m0) * ldb;
        const auto rc = __builtin_amdgcn_make_buffer_rsrc(C + static_cast<size_t>(m0) * ldc + n0, 0, range, 0x00020000);
        const auto rres = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<bf16_t*>(EPI == EPI_RESIDUAL ? residual + static_cast<size_t>(m0) * ldc + n0 : C), 0,
            EPI == EPI_RESIDUAL ? range : 0u, 0x00020000);
        const auto rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(bias != nullptr ? bias + n0 : C), 0,
                                                          bias != nullptr ? static_cast<uint32_t>(N - n0) * 2 : 0u,
                                                          0x00020000);
        const uint32_t rowv = static_cast<uint32_t>(wm * 128 + ml) * ldb;
        float xsr[NB];
#pragma unroll
        for (int j = 0; j < NB; ++j) xsr[j] = x_scale[mcl(row(j))];
        auto widen8 = [](const u32x4& w, float (&o)[8]) {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            o[2 * e] = __uint_as_float(w[e] << 16), o[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
        };
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) {
          uint32_t colv[2];
#pragma unroll
          for (int pp = 0; pp < 2; ++pp) {
            const int cl = wn * 128 + nb * 32 + 8 * (2 * pp + h);
            colv[pp] = n0 + cl < N ? static_cast<uint32_t>(cl) * 2 : 0x80000000u;
          }
          f32x4 wsq[NG];
#pragma unroll
          for (int g = 0; g < NG; ++g) wsq[g] = *reinterpret_cast<const f32x4*>(w_scale + ncl(col(nb * NG + g)));
          u32x4 rq[NB][2], bq[2];
#pragma unroll
          for (int pp = 0; pp < 2; ++pp) {
            bq[pp] = __builtin_amdgcn_raw_buffer_load_b128(rb, colv[pp], 0, 0);
            if constexpr (EPI == EPI_RESIDUAL) {
#pragma unroll
              for (int j = 0; j < NB; ++j)
                rq[j][pp] = __builtin_amdgcn_raw_buffer_load_b128(
                    rres, rowv + colv[pp] + static_cast<uint32_t>(j * MB) * ldb, 0, 0);
            }
          }
#pragma unroll
          for (int j = 0; j < NB; ++j) {
            const auto blk = value(nb, j);
#pragma unroll
            for (int pp = 0; pp < 2; ++pp) {
              const int g = 2 * pp;
              float o[8], add[8];
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const auto r = __builtin_amdgcn_permlane32_swap(
                    __float_as_uint(blk[4 * g + e] * (xsr[j] * wsq[g][e])),
                    __float_as_uint(blk[4 * (g + 1) + e] * (xsr[j] * wsq[g + 1][e])), false, false);
                o[e] = __uint_as_float(r[0]);
                o[4 + e] = __uint_as_float(r[1]);
              }
              widen8(bq[pp], add);
#pragma unroll
              for (int e = 0; e < 8; ++e) o[e] += add[e];
              if constexpr (EPI == EPI_RESIDUAL) {
                widen8(rq[j][pp], add);
#pragma unroll
                for (int e = 0; e < 8; ++e) o[e] += add[e];
              }
              const u32x2 lo = __builtin_bit_cast(u32x2, pack4(o[0], o[1], o[2], o[3]));
              const u32x2 hi = __builtin_bit_cast(u32x2, pack4(o[4], o[5], o[6], o[7]));
              __builtin_amdgcn_raw_buffer_store_b128(u32x4{lo[0], lo[1], hi[0], hi[1]}, rc,
                                                     rowv + colv[pp] + static_cast<uint32_t>(j * MB) * ldb, 0, 0);
            }
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        return;
      }
      load_batch(0, 0);
#pragma unroll
      for (int j0 = 0; j0 < NB; j0 += JG) {
        const int bf = (j0 / JG) & 1;
        if (j0 + JG < NB) load_batch(bf ^ 1, j0 + JG);
#pragma unroll
        for (int jj = 0; jj < JG; ++jj) {
          const int j = j0 + jj, m = row(j);
#pragma unroll
          for (int nb = 0; nb < NB; ++nb) {
            const auto blk = value(nb, j);
#pragma unroll
            for (int g = 0; g < NG; ++g) {
              const int q = nb * NG + g, n = col(q);
              float v[4] = {blk[4 * g], blk[4 * g + 1], blk[4 * g + 2], blk[4 * g + 3]};
              if (bias != nullptr) {
                const u16x4 b = *reinterpret_cast<const u16x4*>(bias + ncl(n));
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] += bf2f(b[e]);
              }
              if constexpr (EPI == EPI_RESIDUAL) {
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] += bf2f(rr[bf][jj][q][e]);
              }
              if (m < M && n < N) st4(C + static_cast<size_t>(m) * ldc + n, pack4(v[0], v[1], v[2], v[3]));
            }
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };

  // accumulator block -> VGPRs through explicit reads: the accumulators then have no use outside
  // asm AGPR operands inside the loop (a plain copy there lets hipcc re-class them and spill)
  auto read_acc = [&](const auto& a) {
    std::remove_cv_t<std::remove_reference_t<decltype(a)>> r;
#pragma unroll
    for (int e = 0; e < (L32 ? 16 : 4); ++e) {
      float v;
      asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(v) : "a"(a[e]));
      r[e] = v;
    }
    return r;
  };
  // the accumulators restart at zero for the next item: MFMAs of zero operands with an inline-0
  // accumulator write them in place (a plain `acc = 0` makes hipcc route the zeros through
  // VGPRs and spill across the loop)
  auto zero_acc = [&]() {
    // (z's VALU writes -> the MFMAs' reads need wait states that hipcc does not insert before
    // inline asm: without them the first MFMAs read stale registers)
    bf16x8 z = {};
    asm volatile("s_nop 4" : "+v"(z));
#pragma unroll
    for (int i = 0; i < NB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        if constexpr (L32)
          asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %1, 0" : "=a"(acc[i][j]) : "v"(z) : "memory");
        else
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %1, 0" : "=a"(acc[i][j]) : "v"(z) : "memory");
      }
  };

  // ---- fp32 parts of a tile (split-K slabs, stream-K segments): per (wave, block, 16-B quarter)
  // 256 floats, lane-major, so a wave's 64 pieces are one contiguous 64 KiB and a piece lands
  // lane-linearly exactly where that lane reads it back.
  constexpr int QPB = L32 ? 4 : 1;  // 16-B quarters per block per lane
  static_assert(NB * NB * QPB == 64, "64 pieces of 1 KiB per wave and part");
  auto piece_off = [&](int i, int j, int qq) {  // this lane's 16 B of block (i, j), quarter qq
    return static_cast<uint32_t>((((wave * NB + i) * NB + j) * QPB + qq) * 1024 + lane * 16);
  };
  // acc += the n parts at byte offsets off_of(k) (k < n) of `srd`: LDS-DMA rounds of 16 pieces
  // per wave into two alternating 16-KiB buffers of this wave (a round in flight while the
  // previous one is added) -- many loads in flight, no VGPRs held for them.  The caller has
  // retired every other use of the wave's LDS region; the parts were stored write-through (sc1)
  // and every load of them is sc1.
  auto add_parts = [&](float* base_ptr, uint32_t bytes, int n, auto off_of) {
    const i32x4 srd = make_srd(base_ptr, bytes);
    const uint32_t lds_w = lds_base + static_cast<uint32_t>(wave) * 16384;
    auto issue = [&](int k, int g, int b) {
      const uint32_t base = off_of(k) + static_cast<uint32_t>(wave * 64 + 16 * g) * 1024;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const uint32_t soff = __builtin_amdgcn_readfirstlane(base + q * 1024);
        const uint32_t m0v = __builtin_amdgcn_readfirstlane(lds_w + b * 65536 + q * 1024);
        asm volatile("s_mov_b32 m0, %3\n\tbuffer_load_dwordx4 %0, %1, %2 offen sc1 lds"
                     :
                     : "v"(static_cast<uint32_t>(lane) * 16), "s"(srd), "s"(soff), "s"(m0v)
                     : "memory", "m0");
      }
    };
    auto consume = [&](int g, int b) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int f = 16 * g + q, i = f / (NB * QPB), j = (f / QPB) % NB, qq = f % QPB;
        const f32x4 v = *reinterpret_cast<const f32x4*>(smem + wave * 16384 + b * 65536 + q * 1024 + lane * 16);
        // plain arithmetic: past the K-loop hipcc moves accumulators between AGPRs and VGPRs
        // under pressure, and its AGPR write right before an asm read of that AGPR gets no
        // wait states (asm reads here returned stale elements: one element of one block, in
        // some launches)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float a;
          asm volatile("s_nop 1\n\tv_accvgpr_read_b32 %0, %1" : "=v"(a) : "a"(acc[i][j][4 * qq + e]));
          a += v[e];
          asm volatile("v_accvgpr_write_b32 %0, %1" : "=a"(acc[i][j][4 * qq + e]) : "v"(a));
        }
      }
      // these reads are done before the round after next refills buffer b
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    };
    if (n > 0) issue(0, 0, 0);
    for (int k = 0; k < n; ++k) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {  // (4 rounds per part: the buffer index g & 1 is static)
        if (g < 3)
          issue(k, g + 1, (g + 1) & 1);
        else if (k + 1 < n)
          issue(k + 1, 0, 0);
        if (g < 3 || k + 1 < n)
          asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // this round landed, the next in flight
        else
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        // (the bytes of an LDS-DMA can land after its vmcnt: a barrier before the reads, as in
        // the reduce-scatter rounds -- every wave of the workgroup runs add_parts)
        asm volatile("s_barrier" ::: "memory");
        consume(g, g & 1);
      }
    }
  };
  // stream-K: the logical workgroup whose range holds unit u; the tile's segments are those of
  // workgroups wg_of(T nk) .. wg_of((T + 1) nk - 1), segment (r, T) stored in part 2 r + (T is
  // r's first tile ? 0 : 1)
  auto wg_of = [&](int u) {
    return static_cast<int>((static_cast<uint32_t>(u + 1) * G - 1) / static_cast<uint32_t>(tiles * nk_all));
  };
  auto nseg = [&](int T) { return wg_of((T + 1) * nk_all - 1) - wg_of(T * nk_all) + 1; };
  auto sk_part = [&](int r, int T) { return static_cast<uint32_t>(2 * r + (T == sk_u0(r) / nk_all ? 0 : 1)) * (BM * BN * 4); };
  // a partial stream-K segment (in the stream): store this wave's fp32 part.  Counting the
  // segments (and reducing) waits for the end of the stream: bookkeeping inside the K-loop's
  // item-end block made hipcc spill the accumulators.
  auto sk_partial = [&](const Geo& g) {
    if constexpr (!L32) {
      // (the lane index re-enters through an opaque move, as in the epilogue: per-lane offsets
      // hoisted out of the K-loop would hold VGPRs across it and spill)
      int ln = lane;
      asm volatile("" : "+v"(ln));
      const uint32_t lane_off = static_cast<uint32_t>(wave * 64 * 1024 + ln * 16);
      const auto rs = __builtin_amdgcn_make_buffer_rsrc(ws, 0, static_cast<uint32_t>(2 * G) * (BM * BN * 4), 0x00020000);
      const uint32_t part = sk_part(r_wg, g.tile);
#pragma unroll
      for (int i = 0; i < NB; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          const auto v = read_acc(acc[i][j]);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs,
                                                 lane_off + static_cast<uint32_t>(i * NB + j) * 1024, part,
                                                 16 /*sc1*/);
          // one block at a time: hoisting every accumulator read above the stores would need
          // the whole tile in VGPRs inside the K-loop (spills)
          __builtin_amdgcn_sched_barrier(0);
        }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  };

  // phase B of stream tile t (W pieces of tile t + 2 = K-tile kt2 of its item).  Past the last
  // tile the pieces go through a zero-range descriptor: no memory traffic, the zeros land in a
  // stage nobody reads -- branch-free, one body (a branch around the pieces, or two copies of
  // the phase, made hipcc spill the accumulators)
  auto phase_b = [&](int t, int kt2, const i32x4& sX, const i32x4& sW, auto sch) {
    using Sch = decltype(sch);
#pragma clang loop unroll(full)
    for (int idx = 0; idx < SLOTS; ++idx) {
      mf(idx, x1, w1);
      if (idx >= Sch::DB0 && (idx - Sch::DB0) % Sch::DBS == 0 && (idx - Sch::DB0) / Sch::DBS < W4_NPB)
        dma(t + 2, kt2, (idx - Sch::DB0) / Sch::DBS + 8, sX, sW);
      if (idx >= Sch::RB0 && (idx - Sch::RB0) % Sch::RBS == 0 && (idx - Sch::RB0) / Sch::RBS < 16)
        read_frag(t + 1, 0, (idx - Sch::RB0) / Sch::RBS, x0, w0);  // tile t+1 (garbage after the last)
    }
  };
  auto run = [&](auto sch) {
    using Sch = decltype(sch);
    int ktc = 0, jc = 0;  // the live item's K-tile count and index
#ifdef W4_STAMPS  // diagnostic build: per-wave cycles in phase A / the wait + barrier / phase B / epilogues
    const uint64_t t_start = __builtin_amdgcn_s_memtime();
    uint64_t cyc_a = 0, cyc_w = 0, cyc_b = 0, cyc_e = 0, t_end = t_start;
#endif
    for (int t = 0; t < total; ++t) {
      advance();  // the DMA cursor to stream tile t + 2
      const bool more = jd < n_items;
      i32x4 sX, sW;
#pragma unroll
      for (int e = 0; e < 4; ++e)
        sX[e] = __builtin_amdgcn_readfirstlane(more ? dX[e] : nullX[e]),
        sW[e] = __builtin_amdgcn_readfirstlane(more ? dW[e] : nullW[e]);
#pragma clang loop unroll(full)
      for (int idx = 0; idx < SLOTS; ++idx) {  // phase A
        mf(idx, x0, w0);
        if (idx >= Sch::DA0 && (idx - Sch::DA0) % Sch::DAS == 0 && (idx - Sch::DA0) / Sch::DAS < 8)
          dma(t + 2, ktd, (idx - Sch::DA0) / Sch::DAS, sX, sX);
        if (idx >= Sch::RA0 && (idx - Sch::RA0) % Sch::RAS == 0 && (idx - Sch::RA0) / Sch::RAS < 16)
          read_frag(t, 1, (idx - Sch::RA0) / Sch::RAS, x1, w1);
      }
#ifdef W4_STAMPS
      const uint64_t t_a = __builtin_amdgcn_s_memtime();
#endif
      asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)\n\ts_barrier" ::: "memory");
#ifdef W4_STAMPS
      const uint64_t t_w = __builtin_amdgcn_s_memtime();
      cyc_a += t_a - t_end, cyc_w += t_w - t_a;
#endif
      phase_b(t, ktd, sX, sW, sch);
      // the MFMA D -> read wait states at the end of every K-tile, inside the loop: whatever
      // hipcc then does with the accumulators -- the item-end block's reads, its register
      // shuffles on the loop exit (a copy of a just-written block there read 16-lane rows not
      // yet written) -- comes after them.  (The wave waits here for the MFMA pipe it would wait
      // for at the next phase's barrier anyway.)
      asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
#ifdef W4_STAMPS
      t_end = __builtin_amdgcn_s_memtime();
      cyc_b += t_end - t_w;
#endif
      if (nsplit == 1 && ++ktc == gc.nk) {
        // item done: its epilogue runs while the next item's first two K-tiles land (the MFMA
        // D -> read wait states are behind us: end of the K-tile above)
        if (gc.nk == nk_all)
          epilogue(gc, [&](int i, int j) { return read_acc(acc[i][j]); });
        else
          sk_partial(gc);  // (stream-K: a tile cut by this workgroup's range)
        // a counter wait hipcc sees: none of its epilogue loads is left pending across the back
        // edge (it would otherwise wait for them, i.e. drain everything, at the top of the next
        // K-tile).  The next item's pieces have had the whole epilogue to land.
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) (expcnt / lgkmcnt unconstrained)
        zero_acc();
        ktc = 0;
        if (++jc < n_items) gc = geo(jc);
#ifdef W4_STAMPS
        const uint64_t t_e = __builtin_amdgcn_s_memtime();
        cyc_e += t_e - t_end;
        t_end = t_e;
#endif
      }
    }
#ifdef W4_STAMPS
    if (lane == 0 && blockIdx.x < 4096) {
      uint64_t* st = w4_stamps + (static_cast<size_t>(blockIdx.x) * 4 + wave) * 8;
      st[0] = cyc_a, st[1] = cyc_w, st[2] = cyc_b, st[3] = total;
      st[4] = cyc_e, st[5] = __builtin_amdgcn_s_memtime() - t_start, st[6] = n_items, st[7] = 0;
    }
#endif
  };
  if constexpr (F8) {
    if (wave & 1)
      run(SchedF8Alt{});
    else
      run(SchedF8{});
  } else {
    if (wave & 1)
      run(SchedAlt{});
    else
      run(SchedMain{});
  }
  // every piece (the zero-range ones past the end included) has landed before the wave ends
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  if (sk) {
    if constexpr (!L32) {
      __syncthreads();  // every wave's stream is over: the LDS ring is free for the part rounds
      // this workgroup's first and last item, when partial (straight-line code: a loop around
      // the reduction made hipcc spill)
      auto reduce_item = [&](int j) {
        const Geo gp = geo(j);
        if (gp.nk == nk_all) return;  // a whole tile: its epilogue ran in the stream
        const int T = gp.tile;
        // every wave's part of T is stored (sc1, drained before the stream's end); the
        // workgroup that counts last over the tile's segments sums them -- one decision per
        // workgroup, so add_parts' barriers see all four waves
        __syncthreads();
        int* flag = reinterpret_cast<int*>(smem);
        if (tid == 0) {
          int* cnt = counters + T;
          const int last = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nseg(T) - 1;
          if (last) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          flag[0] = last;
        }
        __syncthreads();
        const int last = flag[0];
        __syncthreads();  // every wave has read the flag before the part rounds overwrite it
        if (!last) return;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        // zeros by VALU writes, not zero_acc's MFMAs: out here hipcc spills and reloads
        // accumulators between the asm statements, and its spill store of an asm MFMA's result
        // gets no wait states (it read some 16-lane rows before the MFMA had written them)
#pragma unroll
        for (int i = 0; i < NB; ++i)
#pragma unroll
          for (int jj = 0; jj < NB; ++jj)
#pragma unroll
            for (int e = 0; e < 4; ++e) asm volatile("v_accvgpr_write_b32 %0, 0" : "=a"(acc[i][jj][e]));
        const int rf = wg_of(T * nk_all), rl = wg_of((T + 1) * nk_all - 1);
        add_parts(ws, static_cast<uint32_t>(2 * G) * (BM * BN * 4), rl - rf + 1,
                  [&](int k) { return sk_part(rf + k, T); });
        Geo g;
        g.tile = T;
        tile_geo(g);
        epilogue(g, [&](int i, int jj) { return acc[i][jj]; });
      };
      if (n_items > 0) reduce_item(0);
      if (n_items > 1) reduce_item(n_items - 1);
    }
    return;
  }
  if (split_k == 1) return;  // (the epilogues ran in the stream)

  // ---- split-K (one item per workgroup): every split stores its fp32 tile write-through (sc1);
  // the last arriver adds the OTHER splits' slabs into its own accumulators and runs the
  // ordinary epilogue.  The slabs come in by LDS-DMA, 16 KiB per wave per round into two
  // alternating LDS buffers (a round in flight while the previous one is added): many loads in
  // flight and no VGPRs held for them.  (Summing through per-block register loads inside the
  // epilogue put ~190 dependent round trips on one CU: ~70 us of a 105-us qkv launch at 704
  // rows, profiles/r5_gemm_feed.)  Slab layout: per (wave, block, 16-B quarter) 256 floats,
  // lane-major, so a wave's 64 pieces are one contiguous 64 KiB and a piece lands lane-linearly
  // exactly where that lane reads it back.
  float* slab = ws + static_cast<size_t>(gc.tile) * split_k * (BM * BN);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(slab, 0, split_k * BM * BN * 4, 0x00020000);
  __syncthreads();  // every wave is past its last ds_read: smem is reusable as the flag slot
  int* flag = reinterpret_cast<int*>(smem);
  auto slab_off = [&](int sp, int i, int j, int qq) {
    return (sp * (BM * BN) + (((wave * NB + i) * NB + j) * QPB + qq) * 256 + lane * 4) * 4;
  };
#pragma unroll
  for (int i = 0; i < NB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int qq = 0; qq < QPB; ++qq) {
        const f32x4 part = {acc[i][j][4 * qq], acc[i][j][4 * qq + 1], acc[i][j][4 * qq + 2], acc[i][j][4 * qq + 3]};
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, part), rs, slab_off(gc.split, i, j, qq), 0,
                                               16 /*sc1*/);
      }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int prev = __hip_atomic_fetch_add(&counters[gc.tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == split_k - 1;
    if (last) __hip_atomic_store(&counters[gc.tile], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag[0] = last;
  }
  __syncthreads();
  const int is_last = flag[0];
  __syncthreads();  // every wave has read the flag before the slab rounds overwrite it
  if (!is_last) return;
  if constexpr (L32) {  // fp8 / 32x32 layout: per-block register loads (its heavier epilogue has
                        // no VGPRs to spare for the round scheme's addressing)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    epilogue(gc, [&](int i, int j) {
      std::remove_reference_t<decltype(acc[0][0])> sum = 0.f;
      for (int sp = 0; sp < split_k; ++sp)
#pragma unroll
        for (int qq = 0; qq < QPB; ++qq) {
          const f32x4 v = __builtin_bit_cast(
              f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, slab_off(sp, i, j, qq), 0, 16 /*sc1*/));
#pragma unroll
          for (int e = 0; e < 4; ++e) sum[4 * qq + e] += v[e];
        }
      return sum;
    });
    return;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // (and every slab load is sc1)
  add_parts(slab, static_cast<uint32_t>(split_k) * BM * BN * 4, split_k - 1, [&](int k) {  // the other splits
    return static_cast<uint32_t>(k < gc.split ? k : k + 1) * (BM * BN * 4);
  });
  epilogue(gc, [&](int i, int j) { return acc[i][j]; });
}

// compute units of the current device (one resident workgroup each: 160 KiB of LDS)
int w4_cus() {
  static int cus[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cus[dev] && hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    cus[dev] = 256;
  return cus[dev] > 0 ? cus[dev] : 256;
}

// stream-K grid: one workgroup per CU, never more than there are K-tile units
int w4_sk_grid(int tiles, int nk_all) { return static_cast<int>(std::min<long long>(w4_cus(), 1ll * tiles * nk_all)); }

template <int EPI, bool F8 = false>
int launch_w4(const void* x, const void* w, const void* bias, const void* res, void* c, float* ws, int* cnt, int M,
              int N, int K, int inter, int split_k, hipStream_t stream, const float* xs = nullptr,
              const float* wsc = nullptr) {
  const int m_tiles = (M + BM - 1) / BM, n_tiles = (N + BN - 1) / BN;
  const int ldc = EPI == EPI_SILU_MUL ? inter : N;
  const int nwg = m_tiles * n_tiles * std::max(split_k, 1);
  // persistent: one workgroup per CU streams its items (split_k == 1), or its range of the
  // tiles x K-tiles units (split_k == 0, stream-K)
  const int grid = split_k == 0 ? w4_sk_grid(m_tiles * n_tiles, K / (F8 ? 128 : BK))
                   : W4_PERSIST && split_k == 1 ? std::min(nwg, w4_cus()) : nwg;
  hipLaunchKernelGGL((gemm_w4_kernel<EPI, F8>), dim3(grid), dim3(256),
                     0, stream, x, w, static_cast<const bf16_t*>(bias), static_cast<const bf16_t*>(res),
                     static_cast<bf16_t*>(c), ws, cnt, M, N, K, ldc, inter, m_tiles, n_tiles, split_k, xs, wsc);
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
// split_k*65536 floats, `counters` = 65536 ints, zeroed before first use (the last arriver of
// each tile leaves its counter zeroed).
// split_k == 0: stream-K (one workgroup per CU over the tiles x K-tiles units): `ws` >=
// bcg_gemm_w4_sk_ws_floats() floats, `counters` >= m_tiles*n_tiles zeroed ints (left zeroed).
BCG_API int bcg_gemm_w4_sk_ws_floats() { return 2 * w4_cus() * BM * BN; }

BCG_API int bcg_gemm_w4(int epi, const void* x, const void* w, const void* bias, const void* residual, void* c,
                        void* ws, void* counters, int M, int N, int K, int inter, int split_k, hipStream_t stream) {
  if (M <= 0 || N <= 0 || N % 16 || K % BK || K <= 0 || split_k < 0 || K / BK < split_k) return -2;
  // 32-bit buffer offsets, rows up to a whole tile past the end included
  if (2ull * (M + BM) * K >= (1ull << 31) || 2ull * (N + BN) * K >= (1ull << 31)) return -2;
  // the output (and residual) offsets, a masked column's 0x80000000 bias included, stay 32-bit
  if (2ull * (M + BM) * (epi == EPI_SILU_MUL ? inter : N) >= (1ull << 31)) return -2;
  if (split_k != 1 && (!ws || !counters)) return -2;
  if (split_k == 0) {  // stream-K: a counter per tile; the kernel's unit arithmetic is 32-bit
    const long long tiles = 1ll * ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
    if (tiles > W4_COUNTERS || tiles * (K / BK) * w4_cus() >= (1ll << 31)) return -2;
  }
  if (split_k > 1 && 1ll * ((M + BM - 1) / BM) * ((N + BN - 1) / BN) > W4_COUNTERS) return -2;
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

// fp8 (e4m3fn) projection: C = x_scale[m] * w_scale[n] * (Xq . Wq^T) (+ bias) (+ residual).
// epi: 0 = store, 2 = residual + result.  K % 128 == 0, K/128 >= split_k; N % 16 == 0 (a partial
// last n-tile is masked); x_scale [M] / w_scale [N] fp32; split-K workspace as bcg_gemm_w4.
BCG_API int bcg_gemm_w4_fp8(int epi, const void* xq, const void* wq, const float* x_scale, const float* w_scale,
                            const void* bias, const void* residual, void* c, void* ws, void* counters, int M, int N,
                            int K, int split_k, hipStream_t stream) {
  if (M <= 0 || N <= 0 || N % 16 || K % 128 || K <= 0 || split_k < 1 || K / 128 < split_k) return -2;
  if (!x_scale || !w_scale) return -2;
  if (1ull * (M + BM) * K >= (1ull << 31) || 1ull * (N + BN) * K >= (1ull << 31)) return -2;
  if (2ull * (M + BM) * N >= (1ull << 31)) return -2;  // 32-bit output offsets (see bcg_gemm_w4)
  if (split_k > 1 && (!ws || !counters)) return -2;
  float* wsf = static_cast<float*>(ws);
  int* cnt = static_cast<int*>(counters);
  switch (epi) {
    case EPI_STORE:
      return launch_w4<EPI_STORE, true>(xq, wq, bias, residual, c, wsf, cnt, M, N, K, 0, split_k, stream, x_scale,
                                        w_scale);
    case EPI_RESIDUAL:
      if (!residual) return -2;
      return launch_w4<EPI_RESIDUAL, true>(xq, wq, bias, residual, c, wsf, cnt, M, N, K, 0, split_k, stream,
                                           x_scale, w_scale);
    default: return -2;
  }
}
