// 256 x 256 x 64 "ping-pong" GEMM on CDNA4 matrix cores (gfx950), fused epilogues.
//
//   C[M, N] = X[M, K] · W[N, K]^T            (bf16 in, fp32 accumulate, bf16 out)
//
// The big-tile sibling of gemm.hip for the projections that are large enough to fill the
// chip with 256 x 256 tiles: prefill chunks (M = 16384) and the wide decode buckets
// (M = 448..768: gate_up, LM head; qkv / o / down with split-K).  SURVEY.md §2.3
// K-GEMM-QKV/O/GU/D/LMH; the reference reaches these GEMMs inside vLLM
// (byzantine_consensus_game/vllm_agent.py:430).
//
// Structure (cdna_hip_programming.md "The 256² 8-phase template", rebuilt here):
//   * one workgroup = 8 waves = 2 groups of 4 (group g owns output rows g*128..+128, wave
//     wc of the group owns columns wc*64..+64): per wave 128 x 64 = 8 x 4 blocks of 16x16,
//     128 accumulator VGPRs;
//   * a K-tile (64 deep) is staged as four 16-KiB "half" slots, each filled by ONE
//     glds pair per thread (`global_load_lds`, 16 B per lane, no VGPR round trip):
//       A-lo = X rows {0..63, 128..191}, A-hi = X rows {64..127, 192..255},
//       B-lo = W rows {wc*64 + 0..31},   B-hi = W rows {wc*64 + 32..63};
//     the LDS holds two K-tiles (128 KiB, one workgroup per CU);
//   * a K-tile is computed in 4 phases of 16 MFMAs (one 64 x 32 quadrant of the wave's
//     tile x 64 of K):  j0: read A-lo + B-lo, MFMA(lo, lo) · j1: read B-hi, MFMA(lo, hi) ·
//     j2: read A-hi, MFMA(hi, hi) · j3: (no reads) MFMA(hi, lo);
//   * ping-pong: group 1 runs one barrier behind group 0, so on every SIMD (one wave of
//     each group) one wave issues its MFMAs while the other issues its LDS reads and its
//     glds -- each phase is   reads -> glds -> counted vmcnt -> s_barrier -> lgkmcnt(0)
//     -> 16 MFMA -> s_barrier;
//   * every phase issues exactly one half-slot load, 6 phases ahead of its first read:
//       j0: B-hi(t+1)   j1: A-hi(t+1)   j2: A-lo(t+2)   j3: B-lo(t+2)
//     and the reads are j0: B-lo(t), j1: B-hi(t), j2: A-hi(t), j3: A-lo(t+1) (4, 4, 8, 8)
//     With loads issued in phase p and the wait before phase r's first barrier covering
//     the loads of phases <= r-4 (vmcnt(8): 4 half-slots in flight per wave), a load is
//     visible to the readers of phase >= p+5 and a slot is refilled >= 2 phases after its
//     last read -- the two orderings the schedule above satisfies with zero slack at
//     B-hi/B-lo (derivation in PERF.md, "ping-pong GEMM");
//   * LDS rows are 128 B with the 16-B chunk c of row r at chunk c ^ ((r >> 1) & 7) (the
//     swizzle of gemm.hip: conflict-free fragment ds_read_b128); glds writes linearly, so
//     the swizzle is applied to each lane's SOURCE address;
//   * the operands are swapped in the MFMA (W fragment as A, X as B) so a lane holds 4
//     consecutive output columns of one row: 8-B stores, gate/up pairs in one lane;
//   * XCD-aware tile order (bijective remap): the m-tiles and K-splits of one n-tile run
//     on one XCD, so each weight byte comes from HBM once;
//   * split-K: fp32 partial tiles stored write-through (sc1), last arriver reduces
//     (as gemm.hip, cdna_hip_programming.md §6 Guideline 16 R1).
//
// fp8 variant (F8; BASELINE config 5's prefill projections): e4m3fn operands, a row-wise
// activation scale and a per-output-channel weight scale applied in the epilogue
//   C[m, n] = xs[m] * ws[n] * sum_k Xq[m, k] Wq[n, k]   (+ bias, + residual).
// A K-tile is then 128 elements in the SAME 128-B LDS rows, i.e. the same LDS-DMA bytes and
// fragment reads per K-tile as bf16; each block's two 16-B fragments (chunks fq and 4 + fq)
// are the 32-byte operand of ONE v_mfma_scale_f32_16x16x128_f8f6f4 (unit E8M0 scales; A and B
// share the lane -> k map, so the permuted k order inside the instruction cancels), which
// takes the cycles of two bf16 16x16x32 MFMAs for 4x their K: twice the FLOPs per K-tile.
#include <type_traits>

#include "common.h"

#ifndef PP_GLDS_IN_MFMA
#define PP_GLDS_IN_MFMA 1  // issue a phase's two glds pieces between its own MFMAs (+5-9 % over the read turn)
#endif
#ifndef PP_BUFFER_LDS
#define PP_BUFFER_LDS 0  // 1: buffer_load ... lds (MUBUF, k offset in soffset): measured 1-3 % slower
#endif
#ifndef PP_PIECE0
#define PP_PIECE0 3  // MFMA index (0..15) after which the phase's first glds piece is issued
#endif
#ifndef PP_PIECE1
#define PP_PIECE1 11
#endif
#ifndef PP_RING
#define PP_RING 10  // 16-KiB half slots in the LDS ring (10 = the whole 160 KiB)
#endif
#ifndef PP_LEAD
#define PP_LEAD (PP_RING - 1)  // a half-tile is loaded PP_LEAD phases before the phase after its read
#endif
#ifndef PP_GROUP_M
#define PP_GROUP_M 8  // m-tiles per tile-order group (L2 reuse of both operands at prefill M)
#endif

namespace {

constexpr int PBM = 256, PBN = 256, PBK = 64;
constexpr int HALF = 128 * 128;  // one half slot: 128 rows x 128 B
// half-tile n = 4 t + kind of K-tile t; kind: A-lo, B-lo, B-hi, A-hi.  Half-tile n is read in
// phase n - 1 (j0: B-lo(t), j1: B-hi(t), j2: A-hi(t), j3: A-lo(t+1)), loaded in phase n - LEAD
// into ring slot n % RING.  A wait before phase r's first barrier covers the loads of phases
// <= r - DEPTH; a load of phase p is then visible to the readers of phase >= p + DEPTH + 1
// (RAW: DEPTH <= LEAD - 2), and a slot is refilled >= 2 phases after its last read (WAR:
// RING >= LEAD + 1).  The fp8 variant reads A-lo(t) in phase j0 beside B-lo(t) (phase n for
// that kind: no A operand is carried across K-tiles, which keeps its 8-register operands in
// place) and so loads one phase later (LEAD - 1; WAR then RING >= LEAD + 2).
enum { K_ALO = 0, K_BLO = 1, K_BHI = 2, K_AHI = 3 };
constexpr int RING = PP_RING, LEAD = PP_LEAD, DEPTH = LEAD - 2;
static_assert(RING >= LEAD + 1 && DEPTH >= 2 && 2 * DEPTH <= 62 && RING * HALF <= 160 * 1024, "ring geometry");
enum Epilogue { EPI_STORE = 0, EPI_SILU_MUL = 1, EPI_RESIDUAL = 2 };
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }
// g * sigmoid(g) with the hardware reciprocal (1 ulp; a true division expands to ~10
// instructions with mode switches per element in the epilogue)
__device__ __forceinline__ float silu(float g) { return g * __builtin_amdgcn_rcpf(1.f + __expf(-g)); }

__device__ __forceinline__ void sbar() {
#ifndef PP_NO_SCHED_BARRIER
  __builtin_amdgcn_sched_barrier(0);
#endif
#ifndef PP_ABL_NOBAR
  __builtin_amdgcn_s_barrier();
#endif
#ifndef PP_NO_SCHED_BARRIER
  __builtin_amdgcn_sched_barrier(0);
#endif
}

template <int EPI, bool F8 = false>
__global__ __launch_bounds__(512, 1) void gemm_pp_kernel(
    const void* __restrict__ Xv, const void* __restrict__ Wv, const bf16_t* __restrict__ bias,
    const bf16_t* __restrict__ residual, bf16_t* __restrict__ C, float* __restrict__ ws,
    int* __restrict__ counters, int M, int N, int K, int ldc, int inter, int m_tiles, int n_tiles,
    int split_k, const float* __restrict__ x_scale, const float* __restrict__ w_scale) {
  static_assert(!F8 || EPI != EPI_SILU_MUL, "fp8: store / residual epilogues");
  constexpr int ESZ = F8 ? 1 : 2;   // bytes per element
  constexpr int KT = 128 / ESZ;     // K elements per K-tile (one 128-B LDS row)
  constexpr int LEAD = F8 ? ::LEAD - 1 : ::LEAD, DEPTH = LEAD - 2;
  static_assert(DEPTH >= 2 && RING >= LEAD + 1 + (F8 ? 1 : 0), "ring geometry");
  const unsigned char* X = static_cast<const unsigned char*>(Xv);
  const unsigned char* W = static_cast<const unsigned char*>(Wv);
  // ONE shared array (a second __shared__ object can make hipcc drain vmcnt before every
  // ds_read: cdna_hip_programming.md "Projection GEMM" item 4a)
  __shared__ __attribute__((aligned(1024))) unsigned char smem[RING * HALF];

  // ---- XCD-aware order: bijective remap, then (n-tile, m-tile, k-split) ----
  const int nwg = m_tiles * n_tiles * split_k;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, rem = nwg & 7;
  const int r_id = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (bid >> 3);
  const int split = r_id % split_k;
  const int tile = r_id / split_k;
  // grouped order: PP_GROUP_M m-tiles x all n-tiles per group, m fastest -- an XCD's ~32
  // resident tiles then cover ~8 m x 4 n (X and W both L2-reused); decode (m_tiles <= 8)
  // degenerates to "the m-tiles of one n-tile together"
  const int grp = tile / (PP_GROUP_M * n_tiles), in_grp = tile % (PP_GROUP_M * n_tiles);
  const int gm = min(m_tiles - grp * PP_GROUP_M, PP_GROUP_M);
  const int m_tile = grp * PP_GROUP_M + in_grp % gm, n_tile = in_grp / gm;
  const int m0 = m_tile * PBM, n0 = n_tile * PBN;
  const int nk_all = K / KT;
  const int kt0 = split * nk_all / split_k;
  const int nk = (split + 1) * nk_all / split_k - kt0;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int g = wave >> 2, wc = wave & 3;
  const int fr = lane & 15, fq = lane >> 4;

  // global row of slot row s (0..127) of each half slot
  auto w_row = [&](int r) {  // r: tile row of W (0..255)
    if constexpr (EPI == EPI_SILU_MUL) {  // 16-row blocks alternate gate / up of the same features
      const int blk = r >> 4;
      const int feat = (n0 >> 1) + (blk >> 1) * 16 + (r & 15);
      return (blk & 1) ? inter + feat : feat;
    } else {
      return min(n0 + r, N - 1);  // clamped rows are never stored
    }
  };
  // each thread stages 2 x 16 B of a half slot: rows (wave*2 + i)*8 + lane/8, chunk slot lane%8
  const int st_r0 = wave * 16 + (lane >> 3);
  const int st_phys = lane & 7;
  uint32_t offA[2][2], offB[2][2];  // [hi][i]: byte offsets of the rows (k offset added per tile)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int s = st_r0 + i * 8;
    const int c = st_phys ^ ((s >> 1) & 7);
#pragma unroll
    for (int hi = 0; hi < 2; ++hi) {
      const int am = min(m0 + (s >> 6) * 128 + hi * 64 + (s & 63), M - 1);
      offA[hi][i] = static_cast<uint32_t>(am) * K * ESZ + c * 16;
      const int bn = w_row((s >> 5) * 64 + hi * 32 + (s & 31));
      offB[hi][i] = static_cast<uint32_t>(bn) * K * ESZ + c * 16;
    }
  }
  const int nhalf = 4 * nk;  // half-tiles of this workgroup's K range
  // buffer descriptors (byte ranges < 4 GiB: checked by the host wrapper)
  const __amdgpu_buffer_rsrc_t rsX = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(X), 0,
                                                                       static_cast<uint32_t>(M) * K * ESZ, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsW = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<unsigned char*>(W), 0, static_cast<uint32_t>(EPI == EPI_SILU_MUL ? 2 * inter : N) * K * ESZ,
      0x00020000);
  // glds piece i of half-tile n (kind = n & 3, K-tile n >> 2) into ring slot `slot`
  auto load_piece = [&](int n, int kind, int slot, int i) {
#ifdef PP_ABL_NOLOAD
    if (n >= 8) return;
#endif
    unsigned char* dst = smem + slot * HALF + wave * 2048 + i * 1024;
    const uint32_t k0 = (kt0 + (n >> 2)) * 128;  // bytes
    const uint32_t* off = kind == K_ALO ? offA[0] : kind == K_AHI ? offA[1] : kind == K_BLO ? offB[0] : offB[1];
    if constexpr (PP_BUFFER_LDS) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds((kind == K_ALO || kind == K_AHI) ? rsX : rsW,
                                               (__attribute__((address_space(3))) void*)dst, 16, off[i], k0,
                                               0, 0);
    } else {
      const unsigned char* base = (kind == K_ALO || kind == K_AHI) ? X : W;
      __builtin_amdgcn_global_load_lds(base + (off[i] + k0), dst, 16, 0, 0);
    }
  };
  auto load_half = [&](int n, int kind, int slot) {
    load_piece(n, kind, slot, 0);
    load_piece(n, kind, slot, 1);
  };

  f32x4 acc[4][8];  // [n-block][m-block]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // [block][k-step]; alo/ahi: A-lo / A-hi fragments (A-lo of tile t+1 is read in phase j3 of
  // tile t, beside that phase's MFMAs on A-hi: per-phase reads 4, 4, 8, 8 instead of 12, 4, 8, 0)
  // (fp8: a block's two fragments are the two halves of ONE 8-register MFMA operand, read
  // straight into it -- separate halves cost a copy per MFMA and spill)
  using Frag = std::conditional_t<F8, i32x8, bf16x8[2]>;
  Frag alo[4], ahi[4], blo[2], bhi[2];
  // whole-operand definition (a half-vector store would keep the old operand alive)
  auto put = [](Frag& f, bf16x8 v0, bf16x8 v1) {
    if constexpr (F8) {
      f = __builtin_shufflevector(__builtin_bit_cast(i32x4, v0), __builtin_bit_cast(i32x4, v1), 0, 1, 2, 3, 4, 5,
                                  6, 7);
    } else {
      f[0] = v0;
      f[1] = v1;
    }
  };
  auto read_a = [&](int t, int slot, Frag (&a)[4]) {
#ifdef PP_ABL_NOREAD
    if (t >= 1) return;
#endif
    const unsigned char* base = smem + slot * HALF;
#pragma unroll
    for (int mb = 0; mb < 4; ++mb) {
      const int r = g * 64 + mb * 16 + fr;
      put(a[mb], *reinterpret_cast<const bf16x8*>(base + r * 128 + swz(r, fq) * 16),
          *reinterpret_cast<const bf16x8*>(base + r * 128 + swz(r, 4 + fq) * 16));
    }
  };
  auto read_b = [&](int t, int slot, Frag (&b)[2]) {
#ifdef PP_ABL_NOREAD
    if (t >= 1) return;
#endif
    const unsigned char* base = smem + slot * HALF;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int r = wc * 32 + nb * 16 + fr;
      put(b[nb], *reinterpret_cast<const bf16x8*>(base + r * 128 + swz(r, fq) * 16),
          *reinterpret_cast<const bf16x8*>(base + r * 128 + swz(r, 4 + fq) * 16));
    }
  };
  // 16 MFMAs of one quadrant; with PP_GLDS_IN_MFMA the phase's two glds pieces (K-tile lt,
  // half lslot; lt < 0: none) go between them, where the wave waits on the MFMA pipe anyway
  auto mfma = [&](int nh, int mh, const Frag (&a)[4], const Frag (&b)[2], int ln, int lkind,
                  int lslot) {
#ifndef PP_NO_SETPRIO
    __builtin_amdgcn_s_setprio(1);
#endif
    if constexpr (F8) {  // 8 block-scaled K = 128 MFMAs, each over both 16-B fragments of a block
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
#pragma unroll
        for (int mb = 0; mb < 4; ++mb) {
          // formats 0/0 = e4m3 x e4m3; E8M0 scale 127 = 1.0 for both operands
          acc[nh * 2 + nb][mh * 4 + mb] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
              b[nb], a[mb], acc[nh * 2 + nb][mh * 4 + mb], 0, 0, 0, 127, 0, 127);
          if constexpr (PP_GLDS_IN_MFMA) {
            const int idx = nb * 4 + mb;
            if (idx == PP_PIECE0 / 2 || idx == PP_PIECE1 / 2) {
              __builtin_amdgcn_sched_barrier(0);
              if (ln >= 0) load_piece(ln, lkind, lslot, idx == PP_PIECE1 / 2);
              __builtin_amdgcn_sched_barrier(0);
            }
          }
        }
    } else {
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int nb = 0; nb < 2; ++nb)
#pragma unroll
          for (int mb = 0; mb < 4; ++mb) {
            acc[nh * 2 + nb][mh * 4 + mb] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[nb][s], a[mb][s], acc[nh * 2 + nb][mh * 4 + mb], 0, 0, 0);
            if constexpr (PP_GLDS_IN_MFMA) {
              const int idx = (s * 2 + nb) * 4 + mb;
              if (idx == PP_PIECE0 || idx == PP_PIECE1) {
                __builtin_amdgcn_sched_barrier(0);
                if (ln >= 0) load_piece(ln, lkind, lslot, idx == PP_PIECE1);
                __builtin_amdgcn_sched_barrier(0);
              }
            }
          }
    }
#ifndef PP_NO_SETPRIO
    __builtin_amdgcn_s_setprio(0);
#endif
  };
  // counted wait before the phase's first barrier: loads of phases <= r - DEPTH landed.
  // Loads issued in the read turn (before the wait): 2*DEPTH younger glds may be in flight;
  // loads issued among the MFMAs (after the wait): the newest are phase r-1's, 2*(DEPTH-1).
  auto vm_wait = [&](bool full_window) {
    if (full_window) {
      if constexpr (PP_GLDS_IN_MFMA) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (DEPTH - 1)) : "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * DEPTH) : "memory");
      }
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  };
  // one phase: [read turn done by the caller] wait, barrier, MFMAs (+ this phase's load), barrier
  auto phase = [&](bool window, int nh, int mh, const Frag (&a)[4], const Frag (&b)[2], int ln,
                   int lkind, int lslot) {
    if constexpr (!PP_GLDS_IN_MFMA) {
      if (ln >= 0) load_half(ln, lkind, lslot);
    }
    vm_wait(window);
    sbar();  // pre-barrier
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    mfma(nh, mh, a, b, PP_GLDS_IN_MFMA ? ln : -1, lkind, lslot);
    sbar();  // post-barrier
  };

  // ---- prologue: half-tiles 0..LEAD-1 (phases -LEAD..-1) ----
#pragma unroll
  for (int n = 0; n < LEAD; ++n)
    if (n < nhalf) load_half(n, n & 3, n);  // slot n (n < LEAD < RING)
  if (nhalf >= LEAD) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (LEAD - 2)) : "memory");  // half-tiles 0, 1 landed
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  sbar();
  if (g == 1) sbar();  // group 1 runs one barrier behind group 0
  if constexpr (!F8) read_a(0, 0, alo);  // A-lo(0) = half-tile 0, slot 0 ("phase -1")

  int ls = LEAD % RING, rs = 1;  // ring slots of the next load (n = p + LEAD) and read (n = p + 1)
  auto bump = [](int& x) { x = x + 1 == RING ? 0 : x + 1; };
  for (int t = 0; t < nk; ++t) {
    const int p0 = 4 * t;
    // phase p loads half-tile p + LEAD (if any); kinds are compile-time per j
    auto ln = [&](int j) { return p0 + j + LEAD < nhalf ? p0 + j + LEAD : -1; };
    // wait windows: read-turn loads -> phase r has a load; loads among MFMAs -> phase r-1 has one
    auto win = [&](int j) { return (p0 + j + LEAD - (PP_GLDS_IN_MFMA ? 1 : 0)) < nhalf; };
    // j0: read B-lo(t) (fp8: and A-lo(t), the slot before)
    if constexpr (F8) read_a(t, rs == 0 ? RING - 1 : rs - 1, alo);
    read_b(t, rs, blo);
    phase(win(0), 0, 0, alo, blo, ln(0), (0 + LEAD) & 3, ls);
    bump(ls), bump(rs);
    // j1: read B-hi(t)
    read_b(t, rs, bhi);
    phase(win(1), 1, 0, alo, bhi, ln(1), (1 + LEAD) & 3, ls);
    bump(ls), bump(rs);
    // j2: read A-hi(t)
    read_a(t, rs, ahi);
    phase(win(2), 1, 1, ahi, bhi, ln(2), (2 + LEAD) & 3, ls);
    bump(ls), bump(rs);
    // j3: read A-lo(t+1)
    if (!F8 && t + 1 < nk) read_a(t + 1, rs, alo);
    phase(win(3), 0, 1, ahi, blo, ln(3), (3 + LEAD) & 3, ls);
    bump(ls), bump(rs);
  }
  if (g == 0) sbar();  // balance group 1's extra barrier
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- split-K: partial tiles -> workspace (write-through); the last arriver reduces ----
  if (split_k > 1) {
    typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
    float* slab = ws + static_cast<size_t>(tile) * split_k * (PBM * PBN);
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(slab, 0, split_k * PBM * PBN * 4, 0x00020000);
    __syncthreads();  // every wave is past its last ds_read: smem is reusable as the flag slot
    int* flag = reinterpret_cast<int*>(smem);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int off = (split * (PBM * PBN) + ((wave * 4 + i) * 8 + j) * 256 + lane * 4) * 4;
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, acc[i][j]), rs, off, 0, 16 /*sc1*/);
      }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
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
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int off = (sp * (PBM * PBN) + ((wave * 4 + i) * 8 + j) * 256 + lane * 4) * 4;
          acc[i][j] += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16 /*sc1*/));
        }
    }
  }

  // ---- epilogue: lane holds D[n = 4fq + e][m = fr] of block (nb, mb) ----
  if constexpr (!F8) {
    // bf16: buffer-addressed and 16-B wide, as csrc/kernels/gemm_w4.hip: one v_permlane16_swap
    // per value turns the quads of blocks (2p, 2p+1) into 8 contiguous columns per lane (lane
    // row fq: block 2p + (fq & 1), columns 8 (fq >> 1) ..); rows past M fall outside the
    // descriptor's range, a column past N gets an out-of-range offset.  The whole offset rides in
    // the VGPR: only that part is range-checked (an SGPR offset is added after the check, so a
    // row past M carried there would be written).  Half the stores, no per-quad branch.
    typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
    typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
    constexpr bool SILU = EPI == EPI_SILU_MUL;
    // the lane index re-enters through an opaque move: none of the epilogue's per-lane address
    // math is hoisted above the K-loop (it would hold VGPRs across it)
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int fr = ln & 15, fq = ln >> 4;
    const uint32_t ldb = static_cast<uint32_t>(ldc) * 2;
    const uint32_t range = static_cast<uint32_t>(M - m0) * ldb;
    const auto rc = __builtin_amdgcn_make_buffer_rsrc(C + static_cast<size_t>(m0) * ldc + (SILU ? (n0 >> 1) : n0), 0,
                                                      range, 0x00020000);
    const uint32_t rowv = static_cast<uint32_t>(g * 128 + fr) * ldb;
    auto swap_store = [&](int mb, uint32_t colv, const float (&a)[4], const float (&b)[4], const u32x4v& add0,
                          const u32x4v& add1) {
      float o[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a[e]), __float_as_uint(b[e]), false, false);
        o[e] = __uint_as_float(r[0]);
        o[4 + e] = __uint_as_float(r[1]);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint32_t w0 = add0[e >> 1], w1 = add1[e >> 1];
        o[e] += __uint_as_float((e & 1) ? (w0 & 0xffff0000u) : (w0 << 16)) +
                __uint_as_float((e & 1) ? (w1 & 0xffff0000u) : (w1 << 16));
      }
      u16x4 lo, hi;
#pragma unroll
      for (int e = 0; e < 4; ++e) lo[e] = f2bf(o[e]), hi[e] = f2bf(o[4 + e]);
      const u32x2v l2 = __builtin_bit_cast(u32x2v, lo), h2 = __builtin_bit_cast(u32x2v, hi);
      __builtin_amdgcn_raw_buffer_store_b128(u32x4v{l2[0], l2[1], h2[0], h2[1]}, rc,
                                             rowv + colv + static_cast<uint32_t>(mb * 16) * ldb, 0, 0);
    };
    const u32x4v zero = {0, 0, 0, 0};
    if constexpr (SILU) {
      const uint32_t colv = static_cast<uint32_t>(wc * 32 + (fq & 1) * 16 + (fq >> 1) * 8) * 2;
#pragma unroll
      for (int mb = 0; mb < 8; ++mb) {
        float h[2][4];
#pragma unroll
        for (int nh = 0; nh < 2; ++nh)  // (gate, up) block pairs of the same 16 features
#pragma unroll
          for (int e = 0; e < 4; ++e) h[nh][e] = silu(acc[2 * nh][mb][e]) * acc[2 * nh + 1][mb][e];
        swap_store(mb, colv, h[0], h[1], zero, zero);
      }
    } else {
      uint32_t colv[2];
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        const int cl = wc * 64 + (2 * p + (fq & 1)) * 16 + (fq >> 1) * 8;
        colv[p] = n0 + cl < N ? static_cast<uint32_t>(cl) * 2 : 0x80000000u;
      }
      // bias / residual through zero-range descriptors when absent (loads return 0)
      const auto rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(bias != nullptr ? bias + n0 : C), 0,
                                                        bias != nullptr ? static_cast<uint32_t>(N - n0) * 2 : 0u,
                                                        0x00020000);
      const auto rr = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<bf16_t*>(EPI == EPI_RESIDUAL ? residual + static_cast<size_t>(m0) * ldc + n0 : C), 0,
          EPI == EPI_RESIDUAL ? range : 0u, 0x00020000);
      u32x4v bq[2], rq[2][2];
#pragma unroll
      for (int p = 0; p < 2; ++p) {
        bq[p] = __builtin_amdgcn_raw_buffer_load_b128(rb, colv[p], 0, 0);
        rq[0][p] = EPI == EPI_RESIDUAL ? __builtin_amdgcn_raw_buffer_load_b128(rr, rowv + colv[p], 0, 0) : zero;
      }
#pragma unroll
      for (int mb = 0; mb < 8; ++mb) {
        const int cur = mb & 1;
        if (EPI == EPI_RESIDUAL && mb + 1 < 8) {  // the next m-block's residual in flight
#pragma unroll
          for (int p = 0; p < 2; ++p)
            rq[cur ^ 1][p] = __builtin_amdgcn_raw_buffer_load_b128(
                rr, rowv + colv[p] + static_cast<uint32_t>((mb + 1) * 16) * ldb, 0, 0);
        }
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const float a[4] = {acc[2 * p][mb][0], acc[2 * p][mb][1], acc[2 * p][mb][2], acc[2 * p][mb][3]};
          const float b[4] = {acc[2 * p + 1][mb][0], acc[2 * p + 1][mb][1], acc[2 * p + 1][mb][2],
                              acc[2 * p + 1][mb][3]};
          swap_store(mb, colv[p], a, b, bq[p], rq[cur][p]);
        }
      }
    }
    return;
  }
#pragma unroll
  for (int mb = 0; mb < 8; ++mb) {
    const int m = m0 + g * 128 + mb * 16 + fr;
    if (m >= M) continue;
    if constexpr (EPI == EPI_SILU_MUL) {
#pragma unroll
      for (int nh = 0; nh < 2; ++nh) {  // (gate, up) block pairs of the same 16 features
        const int feat = (n0 >> 1) + (wc * 2 + nh) * 16 + 4 * fq;
        u16x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = f2bf(silu(acc[2 * nh][mb][e]) * acc[2 * nh + 1][mb][e]);
        *reinterpret_cast<u16x4*>(C + static_cast<size_t>(m) * ldc + feat) = o;
      }
    } else {
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const int n = n0 + wc * 64 + nb * 16 + 4 * fq;
        if (n >= N) continue;
        float v[4] = {acc[nb][mb][0], acc[nb][mb][1], acc[nb][mb][2], acc[nb][mb][3]};
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

template <int EPI, bool F8 = false>
int launch_pp(const void* x, const void* w, const void* bias, const void* res, void* c, float* ws, int* cnt, int M,
              int N, int K, int inter, int split_k, hipStream_t stream, const float* xs = nullptr,
              const float* wsc = nullptr) {
  const int m_tiles = (M + PBM - 1) / PBM, n_tiles = (N + PBN - 1) / PBN;
  const int ldc = EPI == EPI_SILU_MUL ? inter : N;
  hipLaunchKernelGGL((gemm_pp_kernel<EPI, F8>), dim3(m_tiles * n_tiles * split_k), dim3(512), 0, stream, x, w,
                     static_cast<const bf16_t*>(bias), static_cast<const bf16_t*>(res), static_cast<bf16_t*>(c), ws,
                     cnt, M, N, K, ldc, inter, m_tiles, n_tiles, split_k, xs, wsc);
  return BCG_CHECK_LAUNCH();
}

}  // namespace

// epi: 0 = store (+bias), 1 = silu(gate)*up into [M, inter], 2 = residual + acc.
// Requirements: K % 64 == 0, K/64 >= split_k; N % 16 == 0 (a partial last n-tile is masked);
// EPI 1: N == 2*inter, inter % 128 == 0.  split_k > 1: `ws` >= m_tiles*n_tiles*split_k*65536
// floats, `counters` >= m_tiles*n_tiles zeroed ints (left zeroed).  Pointers 16-B aligned.
BCG_API int bcg_gemm_pp(int epi, const void* x, const void* w, const void* bias, const void* residual, void* c,
                        void* ws, void* counters, int M, int N, int K, int inter, int split_k, hipStream_t stream) {
  if (M <= 0 || N <= 0 || N % 16 || K % PBK || K <= 0 || split_k < 1 || K / PBK < split_k) return -2;
  if (2ull * M * K >= (1ull << 32) || 2ull * N * K >= (1ull << 32)) return -2;  // 32-bit buffer offsets
  // output / residual offsets (a masked column's 0x80000000 bias included) stay 32-bit
  if (2ull * (M + 256) * (epi == EPI_SILU_MUL ? inter : N) >= (1ull << 31)) return -2;
  if (split_k > 1 && (!ws || !counters)) return -2;
  float* wsf = static_cast<float*>(ws);
  int* cnt = static_cast<int*>(counters);
  switch (epi) {
    case EPI_STORE: return launch_pp<EPI_STORE>(x, w, bias, residual, c, wsf, cnt, M, N, K, inter, split_k, stream);
    case EPI_SILU_MUL:
      if (N != 2 * inter || inter % 128) return -2;
      return launch_pp<EPI_SILU_MUL>(x, w, nullptr, nullptr, c, wsf, cnt, M, N, K, inter, split_k, stream);
    case EPI_RESIDUAL:
      if (!residual) return -2;
      return launch_pp<EPI_RESIDUAL>(x, w, bias, residual, c, wsf, cnt, M, N, K, inter, split_k, stream);
    default: return -2;
  }
}

// fp8 (e4m3fn) prefill projection: C = x_scale[m] * w_scale[n] * (Xq . Wq^T) (+ bias) (+ residual).
// epi: 0 = store, 2 = residual + result.  K % 128 == 0, K/128 >= split_k; N % 16 == 0 (a partial
// last n-tile is masked); x_scale [M] / w_scale [N] fp32; split-K workspace as bcg_gemm_pp.
BCG_API int bcg_gemm_pp_fp8(int epi, const void* xq, const void* wq, const float* x_scale, const float* w_scale,
                            const void* bias, const void* residual, void* c, void* ws, void* counters, int M, int N,
                            int K, int split_k, hipStream_t stream) {
  if (M <= 0 || N <= 0 || N % 16 || K % 128 || K <= 0 || split_k < 1 || K / 128 < split_k) return -2;
  if (!x_scale || !w_scale) return -2;
  if (1ull * M * K >= (1ull << 32) || 1ull * N * K >= (1ull << 32)) return -2;  // 32-bit buffer offsets
  if (2ull * (M + 256) * N >= (1ull << 31)) return -2;                          // output offsets
  if (split_k > 1 && (!ws || !counters)) return -2;
  float* wsf = static_cast<float*>(ws);
  int* cnt = static_cast<int*>(counters);
  switch (epi) {
    case EPI_STORE:
      return launch_pp<EPI_STORE, true>(xq, wq, bias, residual, c, wsf, cnt, M, N, K, 0, split_k, stream, x_scale,
                                        w_scale);
    case EPI_RESIDUAL:
      if (!residual) return -2;
      return launch_pp<EPI_RESIDUAL, true>(xq, wq, bias, residual, c, wsf, cnt, M, N, K, 0, split_k, stream, x_scale,
                                           w_scale);
    default: return -2;
  }
}
