// Standalone timing harness for csrc/kernels/gemm_pp.hip / gemm_rs.hip (one variant per binary: build-time
// -D switches, so variants do not perturb each other's codegen -- cdna_hip_programming.md
// §5.4 rule 19).  Random bf16 operands (hash-based, |x| < 1), weights rotated over copies
// that exceed the 256 MiB Infinity Cache, hipEvent timing of back-to-back launches.
//
//   gemm_pp_bench M N K EPI SPLIT [ITERS]   -> one JSON line
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#ifndef GEMM_FN
#define GEMM_FN bcg_gemm_pp  // or bcg_gemm_rs (csrc/kernels/gemm_rs.hip): same contract
#endif
#ifdef W4_STAMPS
extern "C" int bcg_gemm_w4_stamps(void* host, int n);
#endif
extern "C" int GEMM_FN(int epi, const void* x, const void* w, const void* bias, const void* residual, void* c,
                       void* ws, void* counters, int M, int N, int K, int inter, int split_k, hipStream_t stream);
#ifdef BENCH_FP8  // e4m3fn operands through bcg_gemm_w4_fp8 (EPI 0 / 2)
extern "C" int bcg_gemm_w4_fp8(int epi, const void* xq, const void* wq, const float* x_scale, const float* w_scale,
                               const void* bias, const void* residual, void* c, void* ws, void* counters, int M, int N,
                               int K, int split_k, hipStream_t stream);
constexpr size_t ESZ = 1;
#else
constexpr size_t ESZ = 2;
#endif

__global__ void fill_bf16(uint16_t* p, size_t n, uint32_t seed, float scale) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    h *= 0xc2b2ae35u;
    h ^= h >> 16;
    const float v = ((h & 0xffffff) / 16777216.0f * 2.f - 1.f) * scale;
    p[i] = (uint16_t)(__float_as_uint(v) >> 16);
  }
}

// e4m3fn bytes with the exponent field below 1111 (never NaN): (hash & 0x77)
__global__ void fill_fp8(uint8_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 16;
    h *= 0x85ebca6bu;
    h ^= h >> 13;
    p[i] = (uint8_t)((h & 0x77) | ((h >> 8) & 0x80));
  }
}

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e_ = (x);                                              \
    if (e_ != hipSuccess) {                                           \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                        \
    }                                                                 \
  } while (0)

int main(int argc, char** argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: %s M N K EPI SPLIT [ITERS]\n", argv[0]);
    return 2;
  }
  const int M = atoi(argv[1]), N = atoi(argv[2]), K = atoi(argv[3]), epi = atoi(argv[4]), split = atoi(argv[5]);
  const int iters = argc > 6 ? atoi(argv[6]) : 20;
  const size_t wbytes = (size_t)N * K * ESZ;
  const int copies = (int)std::max<size_t>(2, std::min<size_t>(8, ((size_t)1 << 30) / wbytes + 1));
  uint16_t *x, *r, *c;
  std::vector<uint16_t*> w(copies);
  CK(hipMalloc(&x, (size_t)M * K * ESZ));
  CK(hipMalloc(&r, (size_t)M * N * 2));
  CK(hipMalloc(&c, (size_t)M * N * 2));
  hipLaunchKernelGGL(fill_bf16, dim3(1024), dim3(256), 0, 0, r, (size_t)M * N, 2u, 1.f);
#ifdef BENCH_FP8
  float *xs, *wsc;
  CK(hipMalloc(&xs, (size_t)M * 4));
  CK(hipMalloc(&wsc, (size_t)N * 4));
  CK(hipMemset(xs, 0, (size_t)M * 4));
  CK(hipMemset(wsc, 0, (size_t)N * 4));
  hipLaunchKernelGGL(fill_fp8, dim3(1024), dim3(256), 0, 0, (uint8_t*)x, (size_t)M * K, 1u);
#else
  hipLaunchKernelGGL(fill_bf16, dim3(1024), dim3(256), 0, 0, x, (size_t)M * K, 1u, 1.f);
#endif
  for (int i = 0; i < copies; ++i) {
    CK(hipMalloc(&w[i], wbytes));
#ifdef BENCH_FP8
    hipLaunchKernelGGL(fill_fp8, dim3(1024), dim3(256), 0, 0, (uint8_t*)w[i], (size_t)N * K, 3u + i);
#else
    hipLaunchKernelGGL(fill_bf16, dim3(1024), dim3(256), 0, 0, w[i], (size_t)N * K, 3u + i, 0.05f);
#endif
  }
  const int tiles = (M + 255) / 256 * ((N + 255) / 256);
  float* ws = nullptr;
  int* cnt = nullptr;
  // the framework's counter array: 65536 zeroed ints (the W4 reduce-scatter split-K keeps its
  // arrival counters at the top of it)
  if (split != 1) {
    CK(hipMalloc(&cnt, (size_t)65536 * 4));
    CK(hipMemset(cnt, 0, (size_t)65536 * 4));
  }
  if (split > 1)
    CK(hipMalloc(&ws, (size_t)tiles * split * 65536 * 4));
  else if (split == 0)  // W4 stream-K: 2 parts per CU
    CK(hipMalloc(&ws, (size_t)2 * 256 * 65536 * 4));
  auto run = [&](int i) {
    const void* res = epi == 2 ? r : nullptr;
    void* out = epi == 2 ? (void*)r : (void*)c;
#ifdef BENCH_FP8
    return bcg_gemm_w4_fp8(epi, x, w[i % copies], xs, wsc, nullptr, res, out, ws, cnt, M, N, K, split, 0);
#else
    return GEMM_FN(epi, x, w[i % copies], nullptr, res, out, ws, cnt, M, N, K, N / 2, split, 0);
#endif
  };
  for (int i = 0; i < 5; ++i)
    if (run(i)) {
      fprintf(stderr, "launch failed\n");
      return 1;
    }
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < iters; ++i) run(i);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  const double us = ms * 1e3 / iters;
  char extra[512] = "";
#ifdef W4_STAMPS
  {  // per-wave cycles per K-tile of the last launch: medians over the stamped waves, and the
     // share of each wave's lifetime spent outside the K-loop (epilogues, prologue)
    std::vector<uint64_t> st(1 << 17);
    CK(hipDeviceSynchronize());
    if (bcg_gemm_w4_stamps(st.data(), 1 << 17) == 0) {
      const int nw = std::min(tiles * split, 4096) * 4;
      std::vector<double> a, wt, b, e, other;
      for (int i = 0; i < nw; ++i) {
        const uint64_t* s8 = &st[i * 8];
        if (!s8[3]) continue;
        a.push_back((double)s8[0] / s8[3]), wt.push_back((double)s8[1] / s8[3]), b.push_back((double)s8[2] / s8[3]);
        e.push_back((double)s8[4] / s8[6]);
        other.push_back(1.0 - (double)(s8[0] + s8[1] + s8[2]) / s8[5]);
      }
      auto med = [](std::vector<double>& v) {
        if (v.empty()) return 0.0;
        std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
        return v[v.size() / 2];
      };
      snprintf(extra, sizeof extra,
               ", \"cyc_per_ktile\": {\"phaseA\": %.0f, \"wait_barrier\": %.0f, \"phaseB\": %.0f}, "
               "\"cyc_per_epilogue\": %.0f, \"frac_outside_kloop\": %.3f",
               med(a), med(wt), med(b), med(e), med(other));
    }
  }
#endif
  printf("{\"variant\": \"%s\", \"M\": %d, \"N\": %d, \"K\": %d, \"epi\": %d, \"split\": %d, \"us\": %.1f, "
         "\"tflops\": %.1f%s}\n",
         VARIANT_NAME, M, N, K, epi, split, us, 2.0 * M * N * K / us / 1e6, extra);
  return 0;
}
