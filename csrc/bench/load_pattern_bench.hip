// Vector-load cost vs the number of cache rows one instruction touches (tools-only microbenchmark).
//
// Every wave streams its own contiguous 64-KiB slices of a 4-GiB buffer (beyond the Infinity
// Cache) with 16-B loads.  A 4 KiB block = 16 "rows" of 256 B (a paged K-cache token row for
// head_dim 128 bf16) is read in 4 instructions, in one of three lane layouts:
//   0  rows16x64 : lane l -> row l & 15, 16-B chunk (l >> 4) + 4 i   (16 rows x 64 B per load:
//                  the MFMA-operand layout of the decode attention's K loads)
//   1  rows8x128 : lane l -> row (l >> 3) + 8 (i & 1), chunk (l & 7) + 8 (i >> 1)
//   2  rows4x256 : lane l -> row (l >> 4) + 4 i, chunk l & 15   (4 full rows per load)
// Same bytes, same order of blocks; only the rows per instruction differ.  Prints GB/s.
//
//   load_pattern_bench [ITERS]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

template <int PAT>
__global__ __launch_bounds__(256) void stream_kernel(const unsigned char* __restrict__ buf, size_t bytes,
                                                     uint32_t* __restrict__ sink) {
  const int lane = threadIdx.x & 63;
  const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
  const size_t waves = (gridDim.x * (size_t)blockDim.x) >> 6;
  constexpr size_t SLICE = 64 << 10;
  u32x4 acc = {0, 0, 0, 0};
  for (size_t s = wave * SLICE; s < bytes; s += waves * SLICE) {
#pragma unroll 4
    for (size_t blk = 0; blk < SLICE; blk += 4096) {
      const unsigned char* b = buf + s + blk;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        int row, chunk;
        if (PAT == 0) row = lane & 15, chunk = (lane >> 4) + 4 * i;
        else if (PAT == 1) row = (lane >> 3) + 8 * (i & 1), chunk = (lane & 7) + 8 * (i >> 1);
        else row = (lane >> 4) + 4 * i, chunk = lane & 15;
        const u32x4 v = *reinterpret_cast<const u32x4*>(b + row * 256 + chunk * 16);
        acc ^= v;
      }
    }
  }
  if ((acc[0] ^ acc[1] ^ acc[2] ^ acc[3]) == 0x12345678u) sink[0] = 1;  // keeps the loads
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 10;
  const size_t bytes = (size_t)4 << 30;
  unsigned char* buf;
  uint32_t* sink;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(buf, 1, bytes));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const char* names[3] = {"rows16x64", "rows8x128", "rows4x256"};
  for (int round = 0; round < 2; ++round)
    for (int pat = 0; pat < 3; ++pat)
      for (int wpc : {4, 8, 16}) {  // waves per CU
        auto launch = [&]() {
          const dim3 grid(cus * wpc / 4), block(256);
          if (pat == 0) hipLaunchKernelGGL(stream_kernel<0>, grid, block, 0, 0, buf, bytes, sink);
          else if (pat == 1) hipLaunchKernelGGL(stream_kernel<1>, grid, block, 0, 0, buf, bytes, sink);
          else hipLaunchKernelGGL(stream_kernel<2>, grid, block, 0, 0, buf, bytes, sink);
        };
        launch();
        CK(hipDeviceSynchronize());
        hipEvent_t a, b;
        CK(hipEventCreate(&a));
        CK(hipEventCreate(&b));
        CK(hipEventRecord(a, 0));
        for (int i = 0; i < iters; ++i) launch();
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("{\"pattern\": \"%s\", \"waves_per_cu\": %d, \"round\": %d, \"GBps\": %.0f}\n", names[pat], wpc, round,
               bytes * (double)iters / (ms * 1e-3) / 1e9);
      }
  return 0;
}
