// Feed-cost microbenchmark for the 256x256 prefill GEMM (tools-only; timing, not results).
//
// One 256-thread workgroup per CU streams GEMM tiles exactly as gemm_w4.hip does (persistent,
// XCD-remapped, grouped m-tiles, 64-deep K-tiles, one wave per SIMD, 64 AGPR accumulator
// blocks), with the MFMA work fixed (2 phases x 64 v_mfma_f32_16x16x32_bf16 per K-tile) and
// 16 ds_read_b128 per phase.  What varies is how the operand bytes reach the CU:
//
//   LAYOUT 0 (the shipped W4 form: 2 x 2 waves of 128 x 128): X and W K-tiles both by LDS-DMA,
//            NDMA pieces per phase per wave (8 = the full 64 KiB per K-tile per CU)
//   LAYOUT 1 (1 x 4 waves of 256 x 64): X by LDS-DMA (NDMA pieces per phase, 4 = 32 KiB per
//            K-tile per CU), each wave's own W columns straight into VGPRs (NDIR 16-B-per-lane
//            loads per phase, 4 = 32 KiB per K-tile per CU), consumed by the next K-tile's MFMAs.
//            WSHUF 1: W pre-shuffled so one load is 1 KiB contiguous; 0: the natural [N][K]
//            layout, one load = 16 rows x 64 B (the MFMA-fragment shape).
//
// The question it answers: is a K-tile's cost set by the bytes through the CU's load path or by
// the LDS-DMA instructions themselves (~40-60 cycles of issue each, profiles/r4_gemm_w4)?
//
//   feed_bench M N K [ITERS]   -> one JSON line per variant, 2 interleaved rounds
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <cstdint>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__device__ __forceinline__ i32x4 make_srd(const void* base, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  i32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane(static_cast<int>(a & 0xffffffffu));
  r[1] = __builtin_amdgcn_readfirstlane(static_cast<int>(a >> 32) & 0xffff);
  r[2] = __builtin_amdgcn_readfirstlane(static_cast<int>(bytes));
  r[3] = 0x00020000;
  return r;
}

template <int LAYOUT, int NDMA, int NDIR, int WSHUF>
__global__ __launch_bounds__(256, 1) __attribute__((amdgpu_waves_per_eu(1, 1))) void feed_kernel(
    const unsigned char* __restrict__ X, const unsigned char* __restrict__ W, float* __restrict__ sink, int M, int N,
    int K) {
  __shared__ __attribute__((aligned(1024))) unsigned char smem[160 * 1024];
  const int m_tiles = M / 256, n_tiles = N / 256, nwg = m_tiles * n_tiles, G = gridDim.x;
  const int n_items = (nwg - 1 - static_cast<int>(blockIdx.x)) / G + 1;
  const int nk = K / 64;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t row_bytes = K * 2;
  const uint32_t lds_base = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(smem));
  const int fr = lane & 15, fq = lane >> 4;

  // every LDS byte random (bf16 values of X) before the loop, and the DMA pieces land where the
  // fragments are read: all MFMA operands are random data in every variant (zero operands raise
  // the clock the chip holds, cdna_hip_programming.md rule 25)
  for (int o = tid * 16; o < 160 * 1024; o += 256 * 16)
    *reinterpret_cast<i32x4*>(smem + o) = *reinterpret_cast<const i32x4*>(X + o + blockIdx.x * 4096);
  __syncthreads();
  f32x4 acc[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) acc[i] = 0.f;
  bf16x8 xa[16], xb[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) xa[i] = xb[i] = bf16x8{};
  bf16x8 wd[2][8];  // LAYOUT 1: direct W fragments of tiles t (in use) and t + 1 (landing)
#pragma unroll
  for (int i = 0; i < 8; ++i) wd[0][i] = wd[1][i] = bf16x8{};

  for (int it = 0; it < n_items; ++it) {
    const int i = blockIdx.x + it * G;
    const int xcd = i & 7, q = nwg >> 3, rem = nwg & 7;
    const int rid = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (i >> 3);
    const int grp = rid / (8 * n_tiles), in_grp = rid % (8 * n_tiles);
    const int gm = min(m_tiles - grp * 8, 8);
    const int m0 = (grp * 8 + in_grp % gm) * 256, n0 = (in_grp / gm) * 256;
    const i32x4 sX = make_srd(X + static_cast<size_t>(m0) * row_bytes, 256u * row_bytes);
    const i32x4 sW = make_srd(W + static_cast<size_t>(n0) * row_bytes, 256u * row_bytes);
    // DMA piece p of wave w: rows 32 p + 8 w + lane / 8, 16-B chunk lane & 7
    const uint32_t pv = (8 * wave + (lane >> 3)) * row_bytes + (lane & 7) * 16;
    // direct W loads of wave w (LAYOUT 1): its 64 columns n0 + 64 w ..
    //   WSHUF 1: 1-KiB records [64-col group][k-step][block][lane]; 0: rows fr, chunk fq
    const uint32_t wv = WSHUF ? lane * 16 : (64 * wave + fr) * row_bytes + fq * 16;
    const i32x4 sWd = WSHUF ? make_srd(W + static_cast<size_t>(n0 + 64 * wave) * row_bytes, 64u * row_bytes) : sW;
    for (int t0 = 0; t0 < nk; t0 += 2) {
#pragma unroll
     for (int cur = 0; cur < 2; ++cur) {  // (static buffer index: rule 20)
      const int t = t0 + cur;
      const uint32_t kb = __builtin_amdgcn_readfirstlane(t * 128);
#pragma unroll
      for (int ph = 0; ph < 2; ++ph) {
        bf16x8(&xc)[16] = ph ? xb : xa;
        bf16x8(&xn)[16] = ph ? xa : xb;
#pragma unroll
        for (int s = 0; s < 64; ++s) {
          if constexpr (LAYOUT == 0) {
            // 8 x 8 blocks: A = W fragment s >> 3 (xc[8 + ..]), B = X fragment s & 7
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                         : "+a"(acc[s])
                         : "v"(xc[8 + (s >> 3)]), "v"(xc[s & 7])
                         : "memory");
          } else {
            // 16 m-blocks x 4 n-blocks, m-major: A = direct W fragment, B = X fragment s >> 2
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                         : "+a"(acc[s])
                         : "v"(wd[cur][ph * 4 + (s & 3)]), "v"(xc[s >> 2])
                         : "memory");
          }
          if (s % 4 == 1) {  // 16 ds_read_b128 per phase: the next phase's fragments
            const int f = s / 4;
            const int off = ((ph ^ 1) * 32768 + f * 2048 + fr * 128 + (((ph * 4 + fq) ^ ((fr >> 1) & 7)) << 4));
            xn[f] = *reinterpret_cast<const bf16x8*>(smem + off);
          }
          if (NDMA && s % (64 / (NDMA ? NDMA : 1)) == 3) {  // LDS-DMA piece
            const int p = ph * NDMA + s / (64 / NDMA);
            const uint32_t m0v = __builtin_amdgcn_readfirstlane(lds_base + (p & 15) * 4096 + wave * 1024);
            const uint32_t vo = pv + (p & 7) * 32 * row_bytes;
            if (LAYOUT == 0 && (p & 1))
              asm volatile("s_mov_b32 m0, %3\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds"
                           :
                           : "v"(vo), "s"(sW), "s"(kb), "s"(m0v)
                           : "memory", "m0");
            else
              asm volatile("s_mov_b32 m0, %3\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds"
                           :
                           : "v"(vo), "s"(sX), "s"(kb), "s"(m0v)
                           : "memory", "m0");
          }
          if (NDIR && s % (64 / (NDIR ? NDIR : 1)) == 5) {  // direct W load for tile t + 1
            const int j = ph * NDIR + s / (64 / NDIR);
            const int kt = t + 1 < nk ? t + 1 : t;
            uint32_t vo, so;
            if (WSHUF) {
              vo = wv;
              so = __builtin_amdgcn_readfirstlane(((2 * kt + (j >> 2)) * 4 + (j & 3)) * 1024);
            } else {  // block j & 3 (16 columns), k-step j >> 2
              vo = wv + (j & 3) * 16 * row_bytes;
              so = __builtin_amdgcn_readfirstlane(kt * 128 + (j >> 2) * 64);
            }
            asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen"
                         : "=v"(wd[cur ^ 1][j])
                         : "v"(vo), "s"(sWd), "s"(so)
                         : "memory");
          }
        }
        // the loads of the previous phase have landed; this phase's may stay in flight
        if constexpr (NDMA + NDIR > 0) {
          asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"i"(NDMA + NDIR) : "memory");
        } else {
          asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        }
        __builtin_amdgcn_sched_barrier(0);
      }
     }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    float v;
    asm volatile("s_nop 7\n\tv_accvgpr_read_b32 %0, %1" : "=v"(v) : "a"(acc[i][0]));
    s += v;
  }
  if (s == 1.2345f) sink[tid] = s;
}

__global__ void fill_bf16(uint16_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    const float v = ((h & 0xffffff) / 16777216.0f * 2.f - 1.f) * 0.5f;
    p[i] = (uint16_t)(__float_as_uint(v) >> 16);
  }
}

typedef void (*KFn)(const unsigned char*, const unsigned char*, float*, int, int, int);
struct Variant {
  const char* name;
  KFn fn;
};

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 16384, N = argc > 2 ? atoi(argv[2]) : 7168,
            K = argc > 3 ? atoi(argv[3]) : 5120;
  const int iters = argc > 4 ? atoi(argv[4]) : 10;
  if (M % 256 || N % 256 || K % 128) {
    fprintf(stderr, "M, N multiples of 256, K of 128\n");
    return 2;
  }
  const Variant vs[] = {
      {"w4_dma8", feed_kernel<0, 8, 0, 0>},        {"w4_nodma", feed_kernel<0, 0, 0, 0>},
      {"d_dma4_dir4_shuf", feed_kernel<1, 4, 4, 1>}, {"d_dma4_dir4_nat", feed_kernel<1, 4, 4, 0>},
      {"d_dir4_shuf", feed_kernel<1, 0, 4, 1>},     {"d_dma4", feed_kernel<1, 4, 0, 1>},
      {"d_none", feed_kernel<1, 0, 0, 1>},
  };
  unsigned char *x, *w;
  float* sink;
  const size_t xb = (size_t)M * K * 2, wb = (size_t)N * K * 2;
  CK(hipMalloc(&x, xb));
  CK(hipMalloc(&w, wb));
  CK(hipMalloc(&sink, 4096));
  hipLaunchKernelGGL(fill_bf16, dim3(1024), dim3(256), 0, 0, (uint16_t*)x, xb / 2, 1u);
  hipLaunchKernelGGL(fill_bf16, dim3(1024), dim3(256), 0, 0, (uint16_t*)w, wb / 2, 2u);
  CK(hipDeviceSynchronize());
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int nwg = (M / 256) * (N / 256);
  const int grid = nwg < cus ? nwg : cus;
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int round = 0; round < 2; ++round)
    for (const Variant& v : vs) {
      for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(v.fn, dim3(grid), dim3(256), 0, 0, x, w, sink, M, N, K);
      CK(hipGetLastError());
      CK(hipEventRecord(a, 0));
      for (int i = 0; i < iters; ++i) hipLaunchKernelGGL(v.fn, dim3(grid), dim3(256), 0, 0, x, w, sink, M, N, K);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      const double us = ms * 1e3 / iters;
      printf("{\"variant\": \"%s\", \"M\": %d, \"N\": %d, \"K\": %d, \"round\": %d, \"us\": %.1f, \"tflops\": %.0f}\n",
             v.name, M, N, K, round, us, 2.0 * M * N * K / us * 1e-6);
      fflush(stdout);
    }
  return 0;
}
